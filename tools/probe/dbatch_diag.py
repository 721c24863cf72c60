"""Stacked batch-2N D pass vs the two N-image passes.

    python tools/probe/dbatch_diag.py [prec size batch] ...   (default: fp16 512 8)

Per configuration:
  1. layer by layer: D's activations on the stacked fake+real batch vs each half alone;
  2. one backward_D in each form: pred, losses, per-tensor D grads, the D scaler state;
  3. (--traj K) K full steps from the reference init in each form: per step the losses, the D / G
     scaler state and the distance between the two runs' fake_B.
"""
import argparse
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import torch  # noqa: E402

from oracle import dsgan_cpu as O  # noqa: E402
from oracle.recipe import make_params, synth_pair  # noqa: E402


def model(prec, batch):
    import dsgan_hip
    from options.train_options import default_train_opt
    from models import create_model
    dsgan_hip.require_gpu()
    random.seed(20)
    torch.manual_seed(20)
    m = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision=prec, batchSize=batch))
    with torch.no_grad():
        for net, pr in ((m.netG, make_params(O.g_param_spec(), "ref", 1000)),
                        (m.netD, make_params(O.d_param_spec(), "ref", 5000)),
                        (m.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    return m


def d_layers(netD, x):
    from dsgan_hip import functional as HF
    outs = []
    h = x
    for idx, stride, use_in in netD.plan:
        c = netD.model[idx]
        if use_in is None:
            h = HF.conv2d(h, c.weight, c.bias, stride=stride, pad=1)
            outs.append(("conv%d" % idx, h))
        elif use_in:
            y = HF.conv2d(h, c.weight, c.bias, stride=stride, pad=1)
            outs.append(("conv%d" % idx, y))
            h = HF.instance_norm(y, act="lrelu")
            outs.append(("in%d" % idx, h))
        else:
            h = HF.conv2d(h, c.weight, c.bias, stride=stride, pad=1, act="lrelu")
            outs.append(("conv%d" % idx, h))
    return outs


def cmp(a, b):
    a, b = a.double(), b.double()
    d = (a - b).abs()
    return "max|d| %.3e rel %.3e neq %d/%d" % (d.max().item(), (d.norm() / max(b.norm().item(), 1e-30)).item(),
                                               int((a != b).sum()), a.numel())


def run(prec, size, batch, traj):
    from dsgan_hip import functional as HF
    print("=== %s %d^2 batch %d" % (prec, size, batch), flush=True)
    m = model(prec, batch)
    A, B = synth_pair(batch, size, seed=51)
    m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * batch, "B_paths": [""] * batch})
    with torch.no_grad():
        m.forward()
        fake = torch.cat((m.real_A, m.fake_B), 1)
        real = torch.cat((m.real_A, m.real_B), 1)
        st = torch.cat((fake, real), 0).contiguous()
        lf, lr, ls = d_layers(m.netD, fake), d_layers(m.netD, real), d_layers(m.netD, st)
        torch.cuda.synchronize()
        for (n, a), (_, b), (_, s) in zip(lf, lr, ls):
            print("  fwd %-7s fake: %s | real: %s" % (n, cmp(s[:batch], a), cmp(s[batch:], b)), flush=True)
    res = {}
    s0 = m.scaler_D.state.clone() if m.scaler_D is not None else None
    for form in (False, True):
        m.d_batch = form
        m.forward()
        m.set_requires_grad(m.netD, True)
        m.optimizer_D.zero_grad()
        m.backward_D()
        if m.scaler_D is not None:
            m.scaler_D.check(m.flatD.grad)
        torch.cuda.synchronize()
        res[form] = dict(pf=m.pred_fake.detach().clone(), pr=m.pred_real.detach().clone(),
                         lf=float(m.loss_D_fake), lr=float(m.loss_D_real),
                         g={k: p.grad.detach().clone() for k, p in m.netD.named_parameters()},
                         sc=m.scaler_D.state.clone() if m.scaler_D is not None else None)
        if s0 is not None:   # undo the check's state change for the second form
            m.scaler_D.state.copy_(s0)
    a, b = res[False], res[True]
    print("  pred_fake %s   pred_real %s" % (cmp(b["pf"], a["pf"]), cmp(b["pr"], a["pr"])))
    print("  loss_D_fake %.9g / %.9g  loss_D_real %.9g / %.9g" % (a["lf"], b["lf"], a["lr"], b["lr"]))
    for k in a["g"]:
        print("  grad %-16s %s  |g| %.3e" % (k, cmp(b["g"][k], a["g"][k]), a["g"][k].double().norm().item()))
    if a["sc"] is not None:
        print("  scaler two-pass %s stacked %s" % (a["sc"].tolist(), b["sc"].tolist()))
    del m
    torch.cuda.empty_cache()
    if traj:
        runs = []
        for form in (False, True):
            m = model(prec, batch)
            m.d_batch = form
            rows = []
            for i in range(traj):
                A, B = synth_pair(batch, size, seed=100 + i)
                m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * batch, "B_paths": [""] * batch})
                m.optimize_parameters()
                torch.cuda.synchronize()
                rows.append(dict(fake=m.fake_B.detach().float().cpu(),
                                 L=[float(x) for x in (m.loss_G_GAN, m.loss_G_L1, m.loss_D_real, m.loss_D_fake)],
                                 rep=m.nonfinite_report(),
                                 sD=m.scaler_D.get_scale() if m.scaler_D is not None else None,
                                 sG=m.scaler_G.get_scale() if m.scaler_G is not None else None))
            runs.append(rows)
            del m
            torch.cuda.empty_cache()
        for i, (r0, r1) in enumerate(zip(*runs)):
            print("  step %d: fake %s  L %s / %s  rep %s / %s  scale D %s/%s G %s/%s"
                  % (i + 1, cmp(r1["fake"], r0["fake"]), ["%.6g" % x for x in r0["L"]], ["%.6g" % x for x in r1["L"]],
                     r0["rep"], r1["rep"], r0["sD"], r1["sD"], r0["sG"], r1["sG"]), flush=True)
        tgt = (B + 1) / 2
        m0 = O.ms_ssim((runs[0][-1]["fake"] + 1) / 2, tgt).item()
        m1 = O.ms_ssim((runs[1][-1]["fake"] + 1) / 2, tgt).item()
        print("  ms_ssim after %d steps: two-pass %.6f stacked %.6f delta %.2e" % (traj, m0, m1, abs(m0 - m1)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg", nargs="*", default=["fp16", "512", "8"])
    ap.add_argument("--traj", type=int, default=0)
    a = ap.parse_args()
    cfg = a.cfg
    for i in range(0, len(cfg), 3):
        run(cfg[i], int(cfg[i + 1]), int(cfg[i + 2]), a.traj)


if __name__ == "__main__":
    main()
