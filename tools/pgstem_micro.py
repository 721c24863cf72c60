"""PatchGAN stem (pgstem.hip) vs the generic path it replaces, at the bench shape (B=16, 6 -> 32 at
256^2): forward, weight-grad (+ bias), data-grad, each timed alone with HIP events (median of 20).
usage: python tools/pgstem_micro.py [--batch 16] [--size 256]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import torch  # noqa: E402

import dsgan_hip  # noqa: E402
from dsgan_hip import functional as HF  # noqa: E402
from dsgan_hip._lib import call, ptr, stream  # noqa: E402
from dsgan_hip import _lib  # noqa: E402


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--prec", default="bf16")
    a = ap.parse_args()
    dsgan_hip.require_gpu()
    HF.set_precision(a.prec)
    N, Cin, Cout, H, W = a.batch, 6, 32, a.size, a.size
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, Cin, H, W, generator=g).cuda()
    w = (torch.randn(Cout, Cin, 4, 4, generator=g) * 0.05).cuda()
    b = (torch.randn(Cout, generator=g) * 0.05).cuda()
    dy = torch.randn(N, Cout, H // 2, W // 2, generator=g).cuda()
    y = torch.empty(N, Cout, H // 2, W // 2, device="cuda")
    dx = torch.empty_like(x)
    dw = torch.zeros_like(w)
    db = torch.zeros_like(b)
    lib = _lib.load()
    ws = torch.empty(lib.dsgan_pgstem_wgrad_workspace(N, Cin, Cout, H, W), device="cuda")
    xb, yb = x[0].numel(), y[0].numel()
    mb = lambda *ts: sum(t.numel() * 4 for t in ts) / 1e6  # noqa: E731
    rows = []
    rows.append(("stem fwd", tmed(lambda: call("dsgan_pgstem_fwd", ptr(x), xb, ptr(w), ptr(b), ptr(y), yb, N, Cin, Cout,
                                                 H, W, 0.2, stream())), mb(x, y)))
    rows.append(("stem wgrad+db", tmed(lambda: call("dsgan_pgstem_wgrad", ptr(dy), yb, ptr(y), yb, ptr(x), xb, ptr(dw),
                                                      ptr(db), N, Cin, Cout, H, W, 0.2, ptr(ws), ws.numel(),
                                                      stream())), mb(dy, y, x)))
    rows.append(("stem dgrad", tmed(lambda: call("dsgan_pgstem_dgrad", ptr(dy), yb, ptr(y), yb, ptr(w), ptr(dx), xb, N,
                                                   Cin, Cout, H, W, 0.2, 0, stream())), mb(dy, y, dx)))
    HF.PGSTEM[0] = False
    rows.append(("generic fwd", tmed(lambda: HF.conv_fwd_raw(x, w, b, 2, 1, act="lrelu", out=y)), mb(x, y)))
    rows.append(("generic act_bwd", tmed(lambda: HF.act_bwd_raw(dy, y, "lrelu")), mb(dy, y, dy)))
    rows.append(("generic wgrad", tmed(lambda: HF.conv_wgrad_raw(dy, x, dw, 2, 1)), mb(dy, x)))
    rows.append(("generic bias sum", tmed(lambda: HF.channel_sum_raw(dy, db)), mb(dy)))
    rows.append(("generic dgrad", tmed(lambda: HF.conv_dgrad_raw(dy, w, (N, Cin, H, W), 2, 1, out=dx)), mb(dy, dx)))
    HF.PGSTEM[0] = True
    # PatchGAN head (pglast.hip) vs the generic small-channel kernels: 256 -> 1, 4x4 s1 at 31^2
    K, Hh = 256, H // 8 - 1
    xh = torch.randn(N, K, Hh, Hh, generator=g).cuda()
    wh = (torch.randn(1, K, 4, 4, generator=g) * 0.05).cuda()
    bh = torch.zeros(1, device="cuda")
    dyh = torch.randn(N, 1, Hh - 1, Hh - 1, generator=g).cuda()
    yh = torch.empty(N, 1, Hh - 1, Hh - 1, device="cuda")
    dxh = torch.empty_like(xh)
    dwh, dbh = torch.zeros_like(wh), torch.zeros_like(bh)
    for on in (True, False):
        HF.PGLAST[0] = on
        tag = "head" if on else "generic head"
        rows.append((tag + " fwd", tmed(lambda: HF.conv_fwd_raw(xh, wh, bh, 1, 1, out=yh)), mb(xh, yh)))
        rows.append((tag + " dgrad", tmed(lambda: HF.conv_dgrad_raw(dyh, wh, tuple(xh.shape), 1, 1, out=dxh)),
                     mb(dyh, dxh)))
        rows.append((tag + " wgrad", tmed(lambda: HF.conv_wgrad_raw(dyh, xh, dwh, 1, 1, db=dbh)), mb(dyh, xh)))
    HF.PGLAST[0] = True
    for name, us, m in rows:
        print("%-18s %8.1f us  %7.1f MB  %6.0f GB/s" % (name, us, m, m * 1e3 / us))


if __name__ == "__main__":
    main()
