"""PatchGAN 4x4 convs through dsgan_pconv: unsplit vs split-K (dsgan_pconv_ws) at the D shapes, B=16."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
from dsgan_hip._lib import call, ptr, stream
import dsgan_hip
dsgan_hip.require_gpu()
L = dsgan_hip._lib.load()


def timeit(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


for N, K, M, H, s, pad in [(16, 128, 256, 32, 1, 1), (16, 256, 128, 31, 1, 2), (16, 64, 128, 64, 2, 1), (16, 32, 64, 128, 2, 1)]:
    Ho = (H + 2 * pad - 4) // s + 1
    x = torch.randn(N, K, H, H, device="cuda")
    wb = (torch.randn(16 * M * K, device="cuda") * 0.05).bfloat16()
    y = torch.empty(N, M, Ho, Ho, device="cuda")
    nws = L.dsgan_pconv_workspace(N, K, M, Ho, Ho)
    ws = torch.empty(max(nws, 1), device="cuda")
    a = lambda: call("dsgan_pconv_ws", ptr(x), K * H * H, ptr(wb), None, ptr(y), M * Ho * Ho, None, 0, N, K, M, H, H, Ho, Ho,
                     4, 4, s, pad, 3, 0, 0.2, 0, None, 0, stream())
    b = lambda: call("dsgan_pconv_ws", ptr(x), K * H * H, ptr(wb), None, ptr(y), M * Ho * Ho, None, 0, N, K, M, H, H, Ho, Ho,
                     4, 4, s, pad, 3, 0, 0.2, 0, ptr(ws), ws.numel(), stream())
    print("K=%d M=%d H=%d s=%d ws=%d | unsplit %.1f us | split %.1f us" % (K, M, H, s, nws, timeit(a) * 1e3, timeit(b) * 1e3),
          flush=True)
