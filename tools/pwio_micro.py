"""Time dsgan_pw_fwd_io (bf16 weight and activation in, as in the training path) (pwconv1 of the unfused MLP blocks) epilogue variants at the c4/c5 shapes:
gelu + bf16 g + bf16 gelu' (the training path), gelu + bf16 g only, no act bf16 out, no act fp32 out."""
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


for N, K, H, M in [(16, 512, 64, 2048), (16, 1024, 32, 4096), (16, 256, 128, 1024)]:
    P = H * H
    x = torch.randn(N, K, P, device="cuda").bfloat16()
    w = (torch.randn(M, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(M, device="cuda")
    g = torch.empty(N, M, P, device="cuda", dtype=torch.bfloat16)
    gp = torch.empty(N, M, P, device="cuda", dtype=torch.bfloat16)
    y32 = torch.empty(N, M, P, device="cuda")
    v = {
        "gelu+g+gp": lambda: call("dsgan_pw_fwd_io", ptr(w), 1, ptr(x), K * P, 1, ptr(g), M * P, 1, ptr(gp), M * P, 1,
                                  ptr(b), M, K, P, N, 1, 0, 0.2, stream()),
        "gelu+g": lambda: call("dsgan_pw_fwd_io", ptr(w), 1, ptr(x), K * P, 1, ptr(g), M * P, 1, None, 0, 0,
                               ptr(b), M, K, P, N, 1, 0, 0.2, stream()),
        "bf16 out": lambda: call("dsgan_pw_fwd_io", ptr(w), 1, ptr(x), K * P, 1, ptr(g), M * P, 1, None, 0, 0,
                                 ptr(b), M, K, P, N, 0, 0, 0.2, stream()),
        "fp32 out": lambda: call("dsgan_pw_fwd_io", ptr(w), 1, ptr(x), K * P, 1, ptr(y32), M * P, 0, None, 0, 0,
                                 ptr(b), M, K, P, N, 0, 0, 0.2, stream()),
    }
    fl = 2.0 * N * P * M * K
    print("M=%d K=%d P=%d: " % (M, K, P) + " | ".join("%s %.3f ms %.0f TF/s" % (k, t, fl / t / 1e9)
                                                    for k, t in ((k, timeit(f)) for k, f in v.items())), flush=True)
    del x, g, gp, y32
