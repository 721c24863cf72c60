"""wconv.hip weight-grads (split partials + wconv_reduce) at the step's shapes, timed alone with HIP
events (median of 20), with a dw checksum so two library builds can be compared (DSGAN_HIP_LIB).
  ConvTranspose 3x3/s2 weight-grads on the 16-bit IN output grad (dsgan_wconv_xh), G decoder;
  PatchGAN 4x4/s2 weight-grads with the folded bias grad (dsgan_wconv_db), D layers 1-3.
usage: python tools/wconv_micro.py [--batch 16]"""
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
    a = ap.parse_args()
    dsgan_hip.require_gpu()
    HF.set_precision("bf16")
    lib = _lib.load()
    N = a.batch
    g = torch.Generator().manual_seed(0)
    # ConvT (Co, H, Ci): D = x [N][Ci][H/2][W/2] fp32, X = dth [N][Co][H][W] bf16, dw [Ci][Co][3][3]
    for Co, H, Ci in ((512, 32, 1024), (256, 64, 512), (128, 128, 256), (64, 256, 128)):
        Hi = H // 2
        x = torch.randn(N, Ci, Hi, Hi, generator=g).cuda()
        dth = torch.randn(N, Co, H, H, generator=g).to(torch.bfloat16).cuda()
        dw = torch.zeros(Ci, Co, 3, 3, device="cuda")
        ws = torch.empty(lib.dsgan_wconv_workspace(N, Co, Ci, Hi, Hi, 3, 3), device="cuda")

        def run():
            call("dsgan_wconv_xh", ptr(x), x[0].numel(), ptr(dth), dth[0].numel(), ptr(dw), ptr(ws), ws.numel(), N, Co,
                 Ci, H, H, Hi, Hi, 3, 3, 2, 1, stream())
        us = tmed(run)
        dw.zero_()
        run()
        torch.cuda.synchronize()
        print("convT wgrad Co=%4d H=%3d Ci=%4d  %8.1f us   sum %.6e  abs %.6e" % (Co, H, Ci, us, dw.double().sum().item(),
                                                                              dw.double().abs().sum().item()))
    # PatchGAN 4x4 s2 (C -> M at H): D = dy [N][M][H/2][W/2], X = x [N][C][H][W] fp32
    for C, M, H in ((32, 64, 128), (64, 128, 64), (128, 256, 32)):
        Ho = H // 2
        dy = torch.randn(N, M, Ho, Ho, generator=g).cuda()
        x = torch.randn(N, C, H, H, generator=g).cuda()
        dw = torch.zeros(M, C, 4, 4, device="cuda")
        db = torch.zeros(M, device="cuda")
        ws = torch.empty(lib.dsgan_wconv_workspace(N, C, M, Ho, Ho, 4, 4), device="cuda")

        def run():
            call("dsgan_wconv_db", ptr(dy), dy[0].numel(), ptr(x), x[0].numel(), ptr(dw), ptr(db), ptr(ws), ws.numel(),
                 N, C, M, H, H, Ho, Ho, 4, 4, 2, 1, stream())
        us = tmed(run)
        dw.zero_()
        db.zero_()
        run()
        torch.cuda.synchronize()
        print("patch wgrad  C=%4d M=%4d H=%3d   %8.1f us   sum %.6e  abs %.6e" % (C, M, H, us, dw.double().sum().item(),
                                                                              dw.double().abs().sum().item()))


if __name__ == "__main__":
    main()
