"""Time the depthwise conv kernels at the DS-GAN shapes (fwd = also the data-grad)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
from dsgan_hip._lib import call, ptr, stream
import dsgan_hip
dsgan_hip.require_gpu()


def timeit(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


for N, C, H, K in [(16, 3, 256, 7), (16, 128, 256, 7), (16, 256, 128, 7), (16, 64, 128, 7), (16, 512, 64, 7), (16, 1024, 32, 7),
                   (16, 32, 128, 9), (16, 32, 128, 3), (16, 64, 64, 9)]:
    x = torch.randn(N, C, H, H, device="cuda")
    y = torch.empty_like(x)
    w = torch.randn(C, 1, K, K, device="cuda")
    b = torch.randn(C, device="cuda")
    dw = torch.zeros_like(w)
    db = torch.zeros_like(b)
    f = lambda: call("dsgan_dwconv_fwd", ptr(x), C * H * H, ptr(w), ptr(b), ptr(y), C * H * H, N, C, H, H, K, 0, 0, stream())
    dws = torch.empty(dsgan_hip._lib.load().dsgan_dwconv_wgrad_workspace(N, C, H, H, K, 1), device="cuda")
    wg = lambda: call("dsgan_dwconv_wgrad", ptr(y), C * H * H, ptr(x), C * H * H, ptr(dw), ptr(db), N, C, H, H, K,
                      ptr(dws), dws.numel(), stream())
    tf, tw = timeit(f), timeit(wg)
    by = 2 * x.numel() * 4
    print("N=%d C=%4d H=%3d K=%d | fwd %.3f ms %5.0f GB/s | wgrad %.3f ms %5.0f GB/s" % (N, C, H, K, tf, by / tf / 1e6, tw, by / tw / 1e6), flush=True)
