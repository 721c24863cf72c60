"""Time the tiled depthwise weight-grads at the DS-GAN shapes: the 7x7 Block convs and the MidMLKA
four-quarter launch (3/5/7/9 on C/4 channels each)."""
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


out = []
for N, C, H in [(16, 128, 128), (16, 32, 128), (16, 128, 64), (16, 64, 64), (16, 128, 32)]:
    q = C // 4
    x = torch.randn(N, C, H, H, device="cuda"); dy = torch.randn_like(x)
    ws = [torch.zeros(q, 1, k, k, device="cuda") for k in (3, 5, 7, 9)]
    bs = [torch.zeros(q, device="cuda") for _ in range(4)]
    wsp = torch.empty(L.dsgan_dwconv_multi_wgrad_workspace(N, q, H, H), device="cuda")
    f = lambda: call("dsgan_dwconv_multi_wgrad", ptr(dy), C * H * H, ptr(x), C * H * H, ptr(ws[0]), ptr(bs[0]), ptr(ws[1]),
                     ptr(bs[1]), ptr(ws[2]), ptr(bs[2]), ptr(ws[3]), ptr(bs[3]), N, q, H, H, ptr(wsp), wsp.numel(), stream())
    out.append("multi C=%d H=%d %.1f us" % (C, H, timeit(f) * 1e3))
for N, C, H in [(16, 256, 32), (16, 128, 64), (16, 1024, 32), (16, 512, 64), (16, 64, 128), (16, 128, 256)]:
    K = 7
    x = torch.randn(N, C, H, H, device="cuda"); dy = torch.randn_like(x)
    dw = torch.zeros(C, 1, K, K, device="cuda"); db = torch.zeros(C, device="cuda")
    dws = torch.empty(L.dsgan_dwconv_wgrad_workspace(N, C, H, H, K, 1), device="cuda")
    f = lambda: call("dsgan_dwconv_wgrad", ptr(dy), C * H * H, ptr(x), C * H * H, ptr(dw), ptr(db), N, C, H, H, K,
                     ptr(dws), dws.numel(), stream())
    out.append("dw7 C=%d H=%d %.1f us" % (C, H, timeit(f) * 1e3))
print(" | ".join(out), flush=True)
