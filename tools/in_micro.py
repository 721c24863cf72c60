"""InstanceNorm fwd+bwd timing on a 256^2 plane workload (A/B of kernel variants)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
from dsgan_hip import functional as HF
N, C, H = 16, 128, int(sys.argv[1]) if len(sys.argv) > 1 else 256
x = torch.randn(N, C, H, H, device="cuda")
dy = torch.randn_like(x)
for _ in range(3):
    y, m, r = HF.instnorm_raw(x, act="gelu")
    HF.instnorm_bwd_raw(dy, x, None, None, m, r, "gelu", False, False)
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
e[0].record()
for _ in range(10):
    y, m, r = HF.instnorm_raw(x, act="gelu")
e[1].record()
for _ in range(10):
    HF.instnorm_bwd_raw(dy, x, None, None, m, r, "gelu", False, False)
e[2].record()
torch.cuda.synchronize()
f, b = e[0].elapsed_time(e[1]) / 10, e[1].elapsed_time(e[2]) / 10
gb = x.numel() * 4 / 1e9
print("IN %dx%dx%d^2 mode=%s: fwd %.3f ms (%.0f GB/s at 2x), bwd %.3f ms (%.0f GB/s at 3x)" % (
    N, C, H, os.environ.get("DSGAN_IN_BIG", "2"), f, 2 * gb / f * 1e3, b, 3 * gb / b * 1e3))
