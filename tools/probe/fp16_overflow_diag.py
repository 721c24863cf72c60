"""Where does the fp16 G backward overflow?  Replays bench.py's configs[4] quality leg (fp16, 512^2,
batch 8, reference init, pool 0, eager steps: bitwise equal to the graph replay) with every
autograd Function of dsgan_hip.functional probed (tools/nan_diag.py's Probe), and at the first step
whose D or G scaler skipped prints the first non-finite record and the records before it, plus the
largest finite magnitudes of that step's backward.

    python tools/probe/fp16_overflow_diag.py [--d_batch 0|1] [--steps K]
"""
import argparse
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd"), os.path.join(REPO, "tools")]

import torch  # noqa: E402

import nan_diag as ND  # noqa: E402
from oracle import dsgan_cpu as O  # noqa: E402
from oracle.recipe import make_params, synth_pair  # noqa: E402
from options.train_options import default_train_opt  # noqa: E402
from models import create_model  # noqa: E402


def terms(m):
    """The D step as usual, then each G loss term's backward (scaled as the step scales it) into a
    private copy of fake_B: which term's input-grad is non-finite."""
    from dsgan_hip import functional as HF
    m._launch_real_features()
    m.forward()
    m.set_requires_grad(m.netD, True)
    m.optimizer_D.zero_grad()
    m.backward_D()
    m.scaler_D.check(m.flatD.grad)
    m.optimizer_D.step()
    m.set_requires_grad(m.netD, False)
    scale = m.scaler_G.get_scale()
    feats = m._take_real_features()
    tv_coef = m.tv_scale / (320 * 256)
    fns = [("gan", lambda x: m.criterionGAN(m.netD(HF.cat_channels(m.real_A, x)), True) * m.w_gan),
           ("l1", lambda x: HF.l1_loss(x, m.real_B)),
           ("vgg", lambda x: m.vgg.perceptual_l1(x, feats) * m.w_vgg),
           ("tv", lambda x: HF.tv_loss(x, tv_coef) * m.w_tv),
           ("ssim", lambda x: (1 - HF.ssim_affine(m.real_B, x, 0.5, 0.5, 1.0)) * m.w_ss)]
    print("G scale %.0f  w_gan %g w_vgg %g w_tv %g w_ss %g" % (scale, m.w_gan, m.w_vgg, m.w_tv, m.w_ss), flush=True)
    for name, f in fns:
        ND.PR.rec, ND.PR.first = [], None
        x = m.fake_B.detach().clone().requires_grad_()
        with HF.deferred_splits():
            loss = f(x)
            (loss * scale).backward()
        torch.cuda.synchronize()
        g = x.grad
        fin = torch.isfinite(g)
        print("  term %-5s loss %.6g  grad max|.| %.4g  non-finite %d of %d  (nan %d)" % (
            name, float(loss), g[fin].abs().max().item() if fin.any() else float("nan"), int((~fin).sum()),
            g.numel(), int(torch.isnan(g).sum())), flush=True)
        for tag, mx, ok in ND.PR.rec:
            print("     %-70s max %.4g%s" % (tag[:70], mx, "" if ok else "  NONFINITE"), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d_batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--terms_at", type=int, default=0,
                    help="at this step (1-based) run the G loss terms' backward one at a time instead of the step")
    a = ap.parse_args()
    print("probe: %d Functions wrapped" % ND._wrap_functions(), flush=True)
    random.seed(20)
    torch.manual_seed(20)
    m = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision="fp16", batchSize=a.batch, cuda_graph=0))
    with torch.no_grad():
        for net, pr in ((m.netG, make_params(O.g_param_spec(), "ref", 1000)),
                        (m.netD, make_params(O.d_param_spec(), "ref", 5000)),
                        (m.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    m.d_batch = bool(a.d_batch)
    ND._wrap_model(m)
    PR = ND.PR
    for i in range(a.steps):
        PR.step, PR.rec, PR.first = i, [], None
        A, B = synth_pair(a.batch, a.size, seed=100 + i)
        m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * a.batch, "B_paths": [""] * a.batch})
        if i + 1 == a.terms_at:
            terms(m)
            break
        m.optimize_parameters()
        torch.cuda.synchronize()
        skG, skD = m.scaler_G.skipped_last(), m.scaler_D.skipped_last()
        # the G backward's records: those after 'flatD params after Adam'
        k0 = next((k for k, r in enumerate(PR.rec) if r[0].startswith("flatD params")), 0)
        bw = [(r[1], k, r[0]) for k, r in enumerate(PR.rec) if k > k0 and r[0].startswith("B ") and r[2]]
        bw.sort(reverse=True)
        print("step %d: skipped G %s D %s  scale G %.0f D %.0f  G-step backward records %d, largest finite:"
              % (i + 1, skG, skD, m.scaler_G.get_scale(), m.scaler_D.get_scale(), len(bw)), flush=True)
        for mx, k, tag in bw[:8]:
            print("     %4d %-70s %.4g" % (k, tag[:70], mx), flush=True)
        if PR.first is not None:
            s, j = PR.first
            print("  FIRST NON-FINITE record %d of %d: %s" % (j, len(PR.rec), PR.rec[j][0]), flush=True)
            for k in range(max(0, j - 30), min(len(PR.rec), j + 4)):
                tag, mx, fin = PR.rec[k]
                print("   %4d %-70s max %.4g%s" % (k, tag[:70], mx, "" if fin else "  NONFINITE"), flush=True)
            names = {id(p): k for k, p in m.netG.named_parameters()}
            bad = [names[id(p)] for p, _, _ in m.flatG.layout if not torch.isfinite(p.grad).all()]
            print("  non-finite G grads (backward order): %d: %s" % (len(bad), bad[:12]), flush=True)
            break


if __name__ == "__main__":
    main()
