"""Calibration of the pointwise GEMM kernels (pwgemm.hip) against the vendor GEMM library on the same
shapes: torch.matmul on ROCm dispatches bf16 batched GEMMs to hipBLASLt.  Measurement only -- the
library is never on the product path.  Shapes: the unfused MLP blocks of one bench step (B = 16),
Y[b] = W X[b] with W [M][K] bf16, X [b][K][P] bf16 (channel-major, the step's layout).

    python tools/gemm_calib.py [--it 20]

Columns: ours with a plain bf16 output, ours with the fp32 output, ours with the gelu pair (bf16
gelu(z) and gelu'(z) out, the step's form for the first GEMM), hipBLASLt bf16 -> bf16, and the
data-grad form (W^T DY, fp32 out) against hipBLASLt on W^T.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import torch  # noqa: E402

import dsgan_hip  # noqa: E402
from dsgan_hip import _lib  # noqa: E402
from dsgan_hip._lib import call, ptr, stream  # noqa: E402
from dsgan_hip import functional as HF  # noqa: E402

B = 16


def timeit(fn, it):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(it):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--it", type=int, default=20)
    a = ap.parse_args()
    dsgan_hip.require_gpu()
    HF.set_precision("bf16")
    lib = _lib.load()
    hd = torch.bfloat16
    print("%-22s | %8s %8s %8s %8s | %8s %8s  (us; TF/s of the best ours / lib in the last columns)" %
          ("M x K @ HW", "ours16", "ours32", "oursGP", "blasLt", "dgr32", "blasLtT"))
    for M, K, H in [(2048, 512, 64), (256, 2048, 64), (4096, 1024, 32), (512, 4096, 32), (1024, 256, 32),
                    (512, 1024, 32), (1024, 2048, 16), (2048, 512, 16)]:
        HW = H * H
        w = (torch.randn(M, K, device="cuda") / K ** 0.5).to(hd)
        wt = w.t().contiguous()     # [K][M]: the data-grad operand of the transposed GEMM
        x = torch.randn(B, K, HW, device="cuda").to(hd)
        dy = torch.randn(B, M, HW, device="cuda").to(hd)
        b = torch.randn(M, device="cuda")
        y16 = torch.empty(B, M, HW, device="cuda", dtype=hd)
        y32 = torch.empty(B, M, HW, device="cuda")
        gp = torch.empty_like(y16)
        dx = torch.empty(B, K, HW, device="cuda")
        n = max(1, lib.dsgan_pw_fd_workspace(0, M, K, HW, B), lib.dsgan_pw_fd_workspace(1, K, M, HW, B))
        ws = torch.empty(n, device="cuda")
        f16 = lambda: call("dsgan_pw_fwd_io_ws", ptr(w), 1, ptr(x), K * HW, 1, ptr(y16), M * HW, 1, None, 0, 0, ptr(b),
                           M, K, HW, B, 0, 0, 0.2, ptr(ws), ws.numel(), stream())
        f32 = lambda: call("dsgan_pw_fwd_io_ws", ptr(w), 1, ptr(x), K * HW, 1, ptr(y32), M * HW, 0, None, 0, 0, ptr(b),
                           M, K, HW, B, 0, 0, 0.2, ptr(ws), ws.numel(), stream())
        fgp = lambda: call("dsgan_pw_fwd_io_ws", ptr(w), 1, ptr(x), K * HW, 1, ptr(y16), M * HW, 1, ptr(gp), M * HW, 1,
                           ptr(b), M, K, HW, B, 1, 0, 0.2, ptr(ws), ws.numel(), stream())
        fdg = lambda: call("dsgan_pw_dgrad_io_ws", ptr(w), 1, ptr(dy), M * HW, 1, ptr(dx), K * HW, 0, None, 0, K, M,
                           HW, B, 0, ptr(ws), ws.numel(), stream())
        lt = lambda: torch.matmul(w, x, out=y16)
        dxl = torch.empty(B, K, HW, device="cuda", dtype=hd)
        ltt = lambda: torch.matmul(wt, dy, out=dxl)
        t = [timeit(fn, a.it) for fn in (f16, f32, fgp, lt, fdg, ltt)]
        fl = 2.0 * B * HW * M * K
        print("%5d x %5d @ %4d^2   | %8.1f %8.1f %8.1f %8.1f | %8.1f %8.1f  (%4.0f / %4.0f TF/s; dgrad %4.0f / %4.0f)"
              % (M, K, H, *t, fl / min(t[0], t[1]) / 1e6, fl / t[3] / 1e6, fl / t[4] / 1e6, fl / t[5] / 1e6),
              flush=True)


if __name__ == "__main__":
    main()
