"""Micro-benchmark of single implicit-GEMM launches (for rocprofv3 --pmc and A/B timing).
usage: gemm_micro.py MODE N Cin H Cout K s [reps] [prec]"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
from dsgan_hip import functional as HF

mode, N, Cin, H, Cout, K, s = sys.argv[1], *map(int, sys.argv[2:8])
reps = int(sys.argv[8]) if len(sys.argv) > 8 else 20
HF.set_precision(sys.argv[9] if len(sys.argv) > 9 else "bf16")
pad = {1: 0, 3: 1, 4: 1}[K]
x = torch.randn(N, Cin, H, H, device="cuda")
w = torch.randn(Cout, Cin, K, K, device="cuda") * 0.05
b = torch.randn(Cout, device="cuda")
Ho = (H + 2 * pad - K) // s + 1
dy = torch.randn(N, Cout, Ho, Ho, device="cuda")
dw = torch.zeros_like(w)
def run():
    if mode == "fwd":
        HF.conv_fwd_raw(x, w, b, s, pad)
    elif mode == "dgrad":
        HF.conv_dgrad_raw(dy, w, tuple(x.shape), s, pad)
    else:
        HF.conv_wgrad_raw(dy, x, dw, s, pad)
for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
fl = 2.0 * N * Cout * Cin * K * K * Ho * Ho
print("%s N=%d Cin=%d H=%d Cout=%d K=%d s=%d: %.3f ms  %.1f TF/s" % (mode, N, Cin, H, Cout, K, s, ms, fl / ms / 1e9))
