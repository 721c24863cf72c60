"""Mismatch statistics of the persistent gelu-pair forward (knob 11) against the one-tile kernel."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
import dsgan_hip
from dsgan_hip import _lib, functional as HF
from dsgan_hip._lib import call, ptr, stream
lib = _lib.load()
for half in ("bf16", "fp16"):
    dsgan_hip.set_precision(half)
    hd = torch.float16 if half == "fp16" else torch.bfloat16
    M, K, HW, NB = 512, 256, 128 * 128, 4
    g0 = torch.Generator(device="cuda").manual_seed(M + K)
    w = (torch.randn(M, K, device="cuda", generator=g0) / K ** 0.5).to(hd)
    b = torch.randn(M, device="cuda", generator=g0)
    x = torch.randn(NB, K, HW, device="cuda", generator=g0).to(hd)
    outs = []
    for pp in (0, 1):
        lib.dsgan_pw_tune(11, pp)
        y = torch.full((NB, M, HW), float("nan"), device="cuda").to(hd)
        gp = torch.full((NB, M, HW), float("nan"), device="cuda").to(hd)
        ws = torch.empty(max(1, lib.dsgan_pw_fd_workspace(0, M, K, HW, NB)), device="cuda")
        call("dsgan_pw_fwd_io_ws", ptr(w), 1, ptr(x), K * HW, 1, ptr(y), M * HW, 1, ptr(gp), M * HW, 1, ptr(b), M, K,
             HW, NB, 1, 0, 0.2, *HF.wsa(ws), stream())
        torch.cuda.synchronize()
        outs.append((y.float(), gp.float()))
    lib.dsgan_pw_tune(11, 0)
    for nm, a, c in (("y", outs[0][0], outs[1][0]), ("gp", outs[0][1], outs[1][1])):
        d = (a != c) & ~(a.isnan() & c.isnan())
        print(half, nm, "mismatch frac %.3e" % d.float().mean().item(), "nan ref", a.isnan().sum().item(),
              "nan pp", c.isnan().sum().item(), "max abs diff %.3e" % (a - c).abs().nan_to_num(0).max().item())
        if d.any():
            idx = d.nonzero()[:5]
            for n_, m_, p_ in idx.tolist():
                print("   at", n_, m_, p_, a[n_, m_, p_].item(), c[n_, m_, p_].item())
