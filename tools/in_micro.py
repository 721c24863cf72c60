"""Time the InstanceNorm kernels (norm_pointwise.hip) at the step's large-plane shapes: forward (fp32
and bf16 output), backward (fp32 dx) and the 16-bit-dx backward of the ConvT nodes.  Each line ends
in a hash of the outputs, so two builds can be compared bit for bit.

    python tools/in_micro.py                          # the in-tree library
    python tools/in_micro.py --libs a.so,b.so,a.so    # builds interleaved, one process each
"""
import hashlib
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2 and sys.argv[1] == "--libs":
    rc = 0
    for lib_path in sys.argv[2].split(","):
        env = dict(os.environ, DSGAN_HIP_LIB=os.path.join(REPO, lib_path))
        rc |= subprocess.run([sys.executable, "-u", os.path.abspath(__file__)], env=env).returncode
    sys.exit(rc)
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import torch  # noqa: E402

import dsgan_hip  # noqa: E402
from dsgan_hip._lib import call, ptr, stream  # noqa: E402

dsgan_hip.require_gpu()
ACT = {None: 0, "gelu": 1}


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def digest(*ts):
    h = hashlib.sha1()
    for t in ts:
        t = t.detach().cpu()
        h.update((t.view(torch.int16) if t.dtype == torch.bfloat16 else t).numpy().tobytes())
    return h.hexdigest()[:10]


print("lib:", os.environ.get("DSGAN_HIP_LIB", "default"), flush=True)
tot = {"fwd": 0.0, "bwd": 0.0, "bwd_h": 0.0}
for N, C, H, act, res in [(16, 128, 256, None, False), (16, 64, 256, None, False), (16, 64, 256, "gelu", True),
                          (16, 64, 256, "gelu", False), (16, 256, 128, None, False), (16, 128, 128, "gelu", True),
                          (16, 512, 64, None, False), (16, 256, 64, "gelu", False), (16, 128, 64, "gelu", True),
                          (16, 1024, 32, None, False), (16, 512, 32, "gelu", False)]:
    HW = H * H
    g = torch.Generator(device="cuda").manual_seed(C + H)
    x = torch.randn(N, C, H, H, device="cuda", generator=g) * 2 + 0.3
    dy = torch.randn(N, C, H, H, device="cuda", generator=g)
    r = torch.randn(N, C, H, H, device="cuda", generator=g) if res else None
    y = torch.empty_like(x)
    mean, rstd = torch.empty(N * C, device="cuda"), torch.empty(N * C, device="cuda")
    dx = torch.empty_like(x)
    dres = torch.empty_like(x) if res else None
    dxh = torch.empty((N, C, H, H), device="cuda", dtype=torch.bfloat16)
    dsum = torch.empty(N * C, device="cuda")
    a = ACT[act]
    fwd = lambda: call("dsgan_instnorm_fwd", ptr(x), C * HW, None, ptr(r), C * HW, ptr(y), C * HW, ptr(mean), ptr(rstd),
                       N, C, HW, a, 0.2, 1e-5, stream())
    bwd = lambda: call("dsgan_instnorm_bwd", ptr(dy), C * HW, ptr(x), C * HW, None, ptr(r), C * HW, ptr(mean), ptr(rstd),
                       ptr(dx), C * HW, ptr(dres), C * HW, None, N, C, HW, a, 0.2, 1e-5, stream())
    bwh = lambda: call("dsgan_instnorm_bwd_h", ptr(dy), C * HW, ptr(x), C * HW, ptr(r), C * HW, ptr(mean), ptr(rstd),
                       ptr(dxh), C * HW, ptr(dsum), ptr(dres), C * HW, N, C, HW, a, 0.2, 1e-5, stream())
    t = [timeit(fwd), timeit(bwd), timeit(bwh)]
    for k, v in zip(("fwd", "bwd", "bwd_h"), t):
        tot[k] += v
    fwd()
    bwd()
    torch.cuda.synchronize()
    d1 = digest(y, dx)
    bwh()
    torch.cuda.synchronize()
    print("C=%4d H=%3d %-5s res=%d | fwd %7.1f  bwd %7.1f  bwd_h %7.1f us | %s %s" %
          (C, H, act, res, *t, d1, digest(dxh, dsum)), flush=True)
print("totals: " + "  ".join("%s %.1f us" % kv for kv in tot.items()), flush=True)
