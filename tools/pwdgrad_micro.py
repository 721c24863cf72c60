"""Time dsgan_pw_dgrad_io (the unfused MLP blocks' pwconv2 data-grad: bf16 W2, fp32 dy, bf16 dz out
multiplied by the bf16 gelu'(z) of the forward) at the c4/c5 shapes, with and without the gp factor."""
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


for N, M, K, H in [(16, 2048, 256, 64), (16, 4096, 512, 32), (16, 2048, 512, 64)]:
    P = H * H
    dy = torch.randn(N, K, P, device="cuda")
    w = (torch.randn(K, M, device="cuda") * 0.05).bfloat16()     # W2 [P_out=K][C4=M]
    gp = torch.rand(N, M, P, device="cuda").bfloat16()
    dz = torch.empty(N, M, P, device="cuda", dtype=torch.bfloat16)
    v = {
        "gp bf16 out": lambda: call("dsgan_pw_dgrad_io", ptr(w), 1, ptr(dy), K * P, 0, ptr(dz), M * P, 1, ptr(gp), M * P,
                                    M, K, P, N, 0, stream()),
        "bf16 out": lambda: call("dsgan_pw_dgrad_io", ptr(w), 1, ptr(dy), K * P, 0, ptr(dz), M * P, 1, None, 0,
                                 M, K, P, N, 0, stream()),
    }
    fl = 2.0 * N * P * M * K
    print("M=%d K=%d P=%d: " % (M, K, P) + " | ".join("%s %.3f ms %.0f TF/s" % (k, t, fl / t / 1e9)
                                                    for k, t in ((k, timeit(f)) for k, f in v.items())), flush=True)
    del dy, gp, dz
