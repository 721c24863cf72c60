"""Time InstanceNorm(+GELU) fwd/bwd at the DS-GAN plane sizes; check against torch fp32.
DSGAN_IN_V4=0/1/2 selects the scalar / float4-streaming / float4-cached kernels."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
import torch.nn.functional as F
from dsgan_hip._lib import call, ptr, stream
import dsgan_hip
dsgan_hip.require_gpu()
GELU = 1


def timeit(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


mode = os.environ.get("DSGAN_IN_V4", "1")
for N, C, H in [(16, 64, 256), (16, 128, 256), (16, 128, 128), (16, 256, 128), (16, 256, 64), (16, 512, 32),
                (16, 1024, 16)]:
    HW = H * H
    x = torch.randn(N, C, H, H, device="cuda") * 0.3 + 0.1
    y = torch.empty_like(x)
    dy = torch.randn_like(x)
    dx = torch.empty_like(x)
    mean = torch.empty(N * C, device="cuda")
    rstd = torch.empty(N * C, device="cuda")
    f = lambda: call("dsgan_instnorm_fwd", ptr(x), C * HW, None, None, 0, ptr(y), C * HW, ptr(mean), ptr(rstd),
                     N, C, HW, GELU, 0.2, 1e-5, stream())
    b = lambda: call("dsgan_instnorm_bwd", ptr(dy), C * HW, ptr(x), C * HW, None, None, 0, ptr(mean), ptr(rstd),
                     ptr(dx), C * HW, None, 0, None, N, C, HW, GELU, 0.2, 1e-5, stream())
    tf = timeit(f)
    tb = timeit(b)
    xr = x.clone().requires_grad_(True)
    yr = F.gelu(F.instance_norm(xr, eps=1e-5))
    yr.backward(dy)
    ef = ((y - yr).abs().max() / yr.abs().max()).item()
    eb = ((dx - xr.grad).abs().max() / xr.grad.abs().max()).item()
    nb = x.numel() * 4
    print("mode %s N=%d C=%4d H=%3d | fwd %.3f ms %5.0f GB/s(3x) err %.1e | bwd %.3f ms %5.0f GB/s(5x) err %.1e"
          % (mode, N, C, H, tf, 3 * nb / tf / 1e6, ef, tb, 5 * nb / tb / 1e6, eb), flush=True)
    del x, y, dy, dx, xr, yr
