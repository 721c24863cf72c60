"""Time the conv weight-grad kernels (wconv.hip) at the DS-GAN shapes vs the HBM floor.
Shapes are in conv terms: x [N,C,H,W] (ConvT: its output grad), dy [N,M,Ho,Wo] (ConvT: its input)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
import dsgan_hip
from dsgan_hip import functional as HF
dsgan_hip.require_gpu()
HF.set_precision("bf16")


def timeit(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


SHAPES = [  # N, C, H, W, M, K, s   (pad 1)
    (16, 64, 256, 256, 128, 3, 2),   # u4 / local.up4
    (16, 128, 128, 128, 256, 3, 2),  # u3
    (16, 256, 64, 64, 512, 3, 2),    # u2
    (16, 512, 32, 32, 1024, 3, 2),   # u1
    (16, 64, 128, 128, 128, 3, 2),   # local.up3
    (16, 32, 128, 128, 64, 4, 2),    # D layer 1
    (16, 64, 64, 64, 128, 4, 2),     # D layer 2
    (16, 128, 32, 32, 256, 4, 1),    # D layer 3
]
for N, C, H, W, M, K, s in SHAPES:
    Ho, Wo = (H + 2 - K) // s + 1, (W + 2 - K) // s + 1
    x = torch.randn(N, C, H, W, device="cuda")
    dy = torch.randn(N, M, Ho, Wo, device="cuda")
    dw = torch.zeros(M, C, K, K, device="cuda")
    t = timeit(lambda: HF.conv_wgrad_raw(dy, x, dw, s, 1))
    by = 4 * (x.numel() + dy.numel())
    fl = 2.0 * N * M * C * K * K * Ho * Wo
    print("C=%4d H=%3d M=%4d K=%d s=%d | %.3f ms  %5.0f GB/s (fp32 floor %.3f ms)  %6.1f TF/s" % (
        C, H, M, K, s, t, by / t / 1e6, by / 6e9, fl / t / 1e9), flush=True)
