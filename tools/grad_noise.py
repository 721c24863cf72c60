"""Diagnostic: per-tensor gradient error of the fp32 HIP step vs the fp64 oracle, repeated to
show run-to-run spread (atomics / reassociation).  Prints the worst err/|g64| ratios."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd"), os.path.join(REPO, "tests")]
import torch
import test_model_gpu as T
from oracle.recipe import synth_pair

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
A, B = synth_pair(2, 64, seed=4)
ratios = {}
s64 = None
poison = os.environ.get("POISON")
for it in range(reps):
    if poison:   # fill the caching allocator's free blocks with NaN: exposes reads of unwritten memory
        junk = [torch.full((1 << 26,), float("nan"), device="cuda") for _ in range(24)]
        del junk
    m, gp, dp = T._model("fp32")
    m.set_input({"A": A, "B": B, "A_paths": ["a"] * 2, "B_paths": ["b"] * 2})
    m.optimize_parameters()
    torch.cuda.synchronize()
    if poison:
        bad = [k for net in (m.netG, m.netD) for k, p in net.named_parameters()
               if p.grad is not None and not torch.isfinite(p.grad).all()]
        print("rep", it, "non-finite grads:", len(bad), bad[:12])
        print("fake_B finite:", bool(torch.isfinite(m.fake_B).all()), "loss_G", m.loss_G.item())
    if s64 is None:
        s32 = T._oracle_step(gp, dp, A, B, torch.float32)
        s64 = T._oracle_step(gp, dp, A, B, torch.float64)
        sens, _ = T.fp32_sensitivity(gp, dp, A, B)
    for net, o32, o64 in ((m.netG, s32.gp, s64.gp), (m.netD, s32.dp, s64.dp)):
        for (k, p), g32, g64 in zip(net.named_parameters(), o32.values(), o64.values()):
            n64 = g64.grad.norm().item()
            err = (p.grad.detach().double().cpu() - g64.grad).norm().item()
            e32 = (g32.grad.double() - g64.grad).norm().item()
            ratios.setdefault(k, []).append((err / max(n64, 1e-30), e32 / max(n64, 1e-30)))
norms = {}
for net, o64 in ((m.netG, s64.gp), (m.netD, s64.dp)):
    for (k, _), g64 in zip(net.named_parameters(), o64.values()):
        norms[k] = g64.grad.norm().item()
ratios = {k: v for k, v in ratios.items() if norms[k] > 1e-5}   # bias-before-IN grads are ~0
sensr = {k: v / max(norms[k], 1e-30) for (_, k), v in sens.items()}
worst = sorted(ratios.items(), key=lambda kv: -max(r[0] for r in kv[1]))[:20]
for k, rs in worst:
    print("%-45s ours %s  oracle32 %.2e  fp32-ulp-spread %.2e" % (k, " ".join("%.2e" % r[0] for r in rs), rs[0][1],
                                                                 sensr.get(k, 0.0)))
