"""Time the fused MLP kernels (mlp.hip) and the bf16 weight-grads at the DS-GAN block shapes."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
from dsgan_hip._lib import call, ptr, stream
import dsgan_hip
from dsgan_hip import functional as HF

dsgan_hip.require_gpu()
N = 16
SHAPES = [("uc4", 128, 64, 256), ("uc3", 256, 128, 128), ("c2", 64, 128, 128), ("c3", 128, 256, 64)]


def timeit(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


for name, C, P, H in SHAPES:
    HW = H * H
    C4 = 4 * C
    h = torch.randn(N, C, H, H, device="cuda")
    dy = torch.randn(N, P, H, H, device="cuda")
    out = torch.zeros(N, P, H, H, device="cuda")
    w1 = (torch.randn(C4, C, device="cuda") / C ** 0.5).bfloat16()
    w2 = (torch.randn(P, C4, device="cuda") / C4 ** 0.5).bfloat16()
    b1 = torch.randn(C4, device="cuda") * 0.1
    b2 = torch.randn(P, device="cuda") * 0.1
    tile = dsgan_hip._lib.load().dsgan_mlp_supported(C, P, HW)
    g = torch.empty(N, C4, H, H, device="cuda", dtype=torch.bfloat16)
    dz = torch.empty_like(g)
    bsum = torch.empty(N * HW // tile, C4, device="cuda")
    dh = torch.empty_like(h)
    gw2 = torch.zeros(P, C4, device="cuda")
    gw1 = torch.zeros(C4, C, device="cuda")
    f = lambda: call("dsgan_mlp_fwd", ptr(h), C * HW, 0, ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(out), P * HW, N, C, P, HW, 1, stream())
    b = lambda: call("dsgan_mlp_bwd", ptr(h), C * HW, 0, ptr(dy), P * HW, ptr(w1), ptr(b1), ptr(w2), ptr(dh), C * HW,
                     ptr(g), ptr(dz), ptr(bsum), N, C, P, HW, stream())
    w2g = lambda: call("dsgan_pw_wgrad_mixed", ptr(dy), P * HW, 0, ptr(g), C4 * HW, 1, ptr(gw2), P, C4, HW, N, ptr(HF._pw_ws(P, C4, HW, N, dy)), stream())
    w1g = lambda: call("dsgan_pw_wgrad_mixed", ptr(dz), C4 * HW, 1, ptr(h), C * HW, 0, ptr(gw1), C4, C, HW, N, ptr(HF._pw_ws(C4, C, HW, N, dz)), stream())
    tf, tb, t2, t1 = timeit(f), timeit(b), timeit(w2g), timeit(w1g)
    fl = 2.0 * N * HW * (C4 * C + C4 * P)
    byf = N * HW * (C + 2 * P) * 4
    byb = N * HW * ((C + P + C) * 4 + 2 * C4 * 2)
    print("%-4s C=%4d P=%4d HW=%6d | fwd %.3f ms (%.0f TF/s, %.0f GB/s) | bwd %.3f ms (%.0f GB/s) | wg2 %.3f wg1 %.3f ms"
          % (name, C, P, HW, tf, fl / tf / 1e9, byf / tf / 1e6, tb, byb / tb / 1e6, t2, t1), flush=True)
