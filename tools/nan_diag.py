"""GPU-only replay of bench.py's quality leg (B=16, 256^2, reference init, bf16, 10 steps): per-step
losses and, with the probe on, the FIRST non-finite tensor of the run.

    python tools/nan_diag.py [arm ...]        arms: base, fold, nosplit, fold_nosplit, guard, fold_guard (the shipped bf16 default has the guard
    on; every arm here sets it explicitly: off unless the arm name says "guard")

  base     the shipped step
  fold     + the PatchGAN 4x4 weight-grad bias fold (HF.WCONV_DB_FOLD: D's conv biases summed from the
           staged dy tiles instead of a channel-sum pass -- another order of the same fp32 sums)
  nosplit  + no split-K for the pointwise FWD / DGRAD launches (dsgan_pw_tune(0, 0): another order
           of G's sums, unrelated to D's biases)
  guard    the bf16 step with the non-finite-gradient guard on (opt.nonfinite_guard)

Probe (DSGAN_PROBE=1, default): every autograd Function of dsgan_hip.functional is wrapped; each
forward output and backward grad is checked with isfinite and its max|.| recorded, and the flat
gradient / parameter buffers are checked after each backward / optimizer step.  The first
non-finite record is printed with the records before it and, when the base arm ran first, the
same records of the base arm at the same step (the graph is identical, so the record index is).
"""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch  # noqa: E402
import dsgan_hip  # noqa: E402
from dsgan_hip import functional as HF, _lib  # noqa: E402
from oracle import dsgan_cpu as O  # noqa: E402
from oracle.recipe import make_params, synth_pair  # noqa: E402
from options.train_options import default_train_opt  # noqa: E402
from models import create_model  # noqa: E402

PROBE = os.environ.get("DSGAN_PROBE", "1") == "1"
STEPS = int(os.environ.get("NAN_DIAG_STEPS", "10"))


class Probe:
    def __init__(self):
        self.rec = []          # (tag, maxabs, finite) of the current step
        self.first = None      # (step, index) of the first non-finite record
        self.step = -1

    def note(self, tag, t):
        if not torch.is_tensor(t) or not t.is_floating_point() or t.numel() == 0:
            return
        m = float(t.detach().abs().max())
        fin = bool(torch.isfinite(t.detach()).all())
        self.rec.append((tag, m, fin))
        if not fin and self.first is None:
            self.first = (self.step, len(self.rec) - 1)


PR = Probe()


def _wrap_functions():
    seen = set()
    for name in dir(HF):
        cls = getattr(HF, name)
        if not (isinstance(cls, type) and issubclass(cls, torch.autograd.Function)) or cls in seen:
            continue
        if cls is torch.autograd.Function:
            continue
        seen.add(cls)
        fwd, bwd = cls.forward, cls.backward

        def f(ctx, *a, __fwd=fwd, __n=name):
            out = __fwd(ctx, *a)
            for i, o in enumerate(out if isinstance(out, tuple) else (out,)):
                PR.note("F %s[%d] %s" % (__n, i, tuple(o.shape) if torch.is_tensor(o) else ""), o)
            return out

        def b(ctx, *g, __bwd=bwd, __n=name):
            out = __bwd(ctx, *g)
            for i, o in enumerate(out if isinstance(out, tuple) else (out,)):
                PR.note("B %s[%d] %s" % (__n, i, tuple(o.shape) if torch.is_tensor(o) else ""), o)
            return out

        cls.forward = staticmethod(f)
        cls.backward = staticmethod(b)
    return len(seen)


def _wrap_model(model):
    bD, bG, oD, oG = model.backward_D, model.backward_G, model.optimizer_D.step, model.optimizer_G.step

    def backward_D(*a):
        bD(*a)
        PR.note("flatD.grad after backward_D", model.flatD.grad)

    def backward_G():
        bG()
        PR.note("flatG.grad after backward_G", model.flatG.grad)

    def stepD():
        oD()
        PR.note("flatD params after Adam", model.flatD.data)

    def stepG():
        oG()
        PR.note("flatG params after Adam", model.flatG.data)

    model.backward_D, model.backward_G = backward_D, backward_G
    model.optimizer_D.step, model.optimizer_G.step = stepD, stepG


def run_arm(arm, base_trace):
    lib = _lib.load()
    HF.WCONV_DB_FOLD = "fold" in arm
    old_split = lib.dsgan_pw_tune(0, 0 if "nosplit" in arm else 1)
    HF.set_precision("bf16")
    random.seed(20)
    torch.manual_seed(20)
    opt = default_train_opt(gpu_ids=[0], pool_size=0, precision="bf16", batchSize=16,
                            nonfinite_guard=1 if "guard" in arm else 0, cuda_graph=0)
    model = create_model(opt)
    gp = make_params(O.g_param_spec(), "ref", 1000)
    dp = make_params(O.d_param_spec(), "ref", 5000)
    with torch.no_grad():
        for net, pr in ((model.netG, gp), (model.netD, dp), (model.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    if PROBE:
        _wrap_model(model)
    PR.first = None
    trace = {}
    for i in range(STEPS):
        PR.step, PR.rec = i, []
        A, B = synth_pair(16, 256, seed=100 + i)
        model.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * 16, "B_paths": [""] * 16})
        model.optimize_parameters()
        torch.cuda.synchronize()
        trace[i] = PR.rec
        vals = dict(G=float(model.loss_G.detach()), D=float(model.loss_D.detach()), L1=float(model.loss_G_L1.detach()),
                    vgg=float(model.loss_vgg.detach()), ssim=float(model.loss_ssim.detach()),
                    fake=float(model.fake_B.detach().float().abs().max()),
                    gG=float(model.flatG.grad.abs().max()), gD=float(model.flatD.grad.abs().max()),
                    pG=float(model.flatG.data.abs().max()), pD=float(model.flatD.data.abs().max()))
        extra = ""
        if model.scaler_G is not None:
            extra = " skippedG=%d skippedD=%d" % (model.scaler_G.skipped_steps(i + 1), model.scaler_D.skipped_steps(i + 1))
        print(arm, i, " ".join("%s=%.4g" % kv for kv in vals.items()) + extra, flush=True)
        if PROBE and PR.first is not None and PR.first[0] == i:
            s, j = PR.first
            print("  FIRST NON-FINITE at step %d record %d of %d: %s" % (s, j, len(PR.rec), PR.rec[j][0]), flush=True)
            ref = base_trace.get(s) if base_trace else None
            for k in range(max(0, j - 25), min(len(PR.rec), j + 3)):
                tag, m, fin = PR.rec[k]
                rm = ("  base %.4g" % ref[k][1]) if ref is not None and k < len(ref) and ref[k][0] == tag else ""
                print("   %4d %-70s max %.4g%s%s" % (k, tag[:70], m, "" if fin else "  NONFINITE", rm), flush=True)
            # the largest magnitudes of this step vs base (growth before the blow-up)
            if ref is not None:
                ratios = []
                for k in range(min(j, len(ref))):
                    if ref[k][0] == PR.rec[k][0] and ref[k][1] > 0:
                        ratios.append((PR.rec[k][1] / ref[k][1], k, PR.rec[k][0], PR.rec[k][1], ref[k][1]))
                ratios.sort(reverse=True)
                print("  largest max|.| ratios vs base before the first non-finite record:", flush=True)
                for r, k, tag, m, rmx in ratios[:12]:
                    print("   %4d %-70s %.4g vs %.4g (x%.3g)" % (k, tag[:70], m, rmx, r), flush=True)
    lib.dsgan_pw_tune(0, old_split)
    del model
    torch.cuda.empty_cache()
    return trace


def main():
    dsgan_hip.require_gpu()
    arms = sys.argv[1:] or ["base", "fold"]
    if PROBE:
        print("probe: %d autograd Functions wrapped" % _wrap_functions(), flush=True)
    base = None
    for arm in arms:
        t = run_arm(arm, base)
        if arm == "base":
            base = t
    HF.WCONV_DB_FOLD = False


if __name__ == "__main__":
    main()
