"""Time the few-channel streaming kernels at the step's 256^2 shapes: the 1x1 weight-grads with a
3-channel side (skinny.hip wgrad_small_pw4) and the 1x1 contractions into <= 16 channels
(pwsmall.hip pw_small_kernel, e.g. the 64 -> 12 data-grad of the c1 block).  Each line ends in a
hash of the output, so two builds compare bit for bit.

    python tools/small_micro.py                          # the in-tree library
    python tools/small_micro.py --libs a.so,b.so,a.so    # builds interleaved, one process each
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
L = dsgan_hip._lib.load()


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


def digest(t):
    return hashlib.sha1(t.detach().cpu().numpy().tobytes()).hexdigest()[:10]


print("lib:", os.environ.get("DSGAN_HIP_LIB", "default"), flush=True)
N, H = 16, 256
P = H * H
tot = 0.0
for Cin, Cout in [(3, 64), (3, 32), (3, 12)]:
    g = torch.Generator(device="cuda").manual_seed(Cout)
    dy = torch.randn(N, Cout, H, H, device="cuda", generator=g)
    x = torch.randn(N, Cin, H, H, device="cuda", generator=g)
    dw = torch.zeros(Cout, Cin, 1, 1, device="cuda")
    ws = torch.empty(max(1, L.dsgan_conv_wgrad_small_workspace(N, Cin, Cout, 1, 1, H, H)), device="cuda")
    f = lambda: call("dsgan_conv_wgrad_small", ptr(dy), Cout * P, ptr(x), Cin * P, ptr(dw), N, Cin, H, H, Cout, 1, 1,
                     1, 0, H, H, ptr(ws), ws.numel(), stream())
    t = timeit(f)
    tot += t
    dw.zero_()
    f()
    torch.cuda.synchronize()
    print("wgrad_small %2d -> %2d | %7.1f us | %s" % (Cin, Cout, t, digest(dw)), flush=True)
for K, M in [(64, 12), (64, 3), (12, 3)]:
    g = torch.Generator(device="cuda").manual_seed(K + M)
    x = torch.randn(N, K, H, H, device="cuda", generator=g)
    w = torch.randn(M, K, device="cuda", generator=g) / K ** 0.5
    y = torch.empty(N, M, H, H, device="cuda")
    f = lambda: call("dsgan_pw_small", ptr(x), K * P, ptr(w), K, 1, None, ptr(y), M * P, None, 0, N, K, M, P, 0, 0,
                     0, 0, 0.2, stream())
    t = timeit(f)
    tot += t
    f()
    torch.cuda.synchronize()
    print("pw_small %2d -> %2d | %7.1f us | %s" % (K, M, t, digest(y)), flush=True)
print("total: %.1f us" % tot, flush=True)
