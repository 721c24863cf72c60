"""The G head conv 64 -> 3, 3x3 s1 p1 at 256^2, B=16 (thin3.hip): forward, data-grad, weight-grad
timed with HIP events (median of 20) against the library DSGAN_HIP_LIB names (A/B of two builds)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import torch  # noqa: E402

import dsgan_hip  # noqa: E402
from dsgan_hip import functional as HF  # noqa: E402


def tmed(fn, n=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dsgan_hip.require_gpu()
    HF.set_precision("bf16")
    N, K, M, H = 16, 64, 3, 256
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, K, H, H, generator=g).cuda()
    w = (torch.randn(M, K, 3, 3, generator=g) * 0.05).cuda()
    b = torch.randn(M, generator=g).cuda()
    dy = torch.randn(N, M, H, H, generator=g).cuda()
    y = torch.empty(N, M, H, H, device="cuda")
    dx = torch.empty_like(x)
    dw = torch.zeros_like(w)
    HF.conv_fwd_raw(x, w, b, 1, 1, out=y)
    HF.conv_dgrad_raw(dy, w, tuple(x.shape), 1, 1, out=dx)
    HF.conv_wgrad_raw(dy, x, dw, 1, 1)
    torch.cuda.synchronize()
    h = [float(t.double().sum()) for t in (y, dx, dw)]
    print("thin3 fwd   %7.1f us" % tmed(lambda: HF.conv_fwd_raw(x, w, b, 1, 1, out=y)))
    print("thin3 dgrad %7.1f us" % tmed(lambda: HF.conv_dgrad_raw(dy, w, tuple(x.shape), 1, 1, out=dx)))
    print("thin3 wgrad %7.1f us" % tmed(lambda: HF.conv_wgrad_raw(dy, x, dw, 1, 1)))
    print("sums %.6e %.6e %.6e" % tuple(h))


if __name__ == "__main__":
    main()
