"""Time dsgan_pconvt (ConvTranspose2d 3x3/s2 forward and the PatchGAN 4x4/s2 data-grad, pconvt.hip)
at the step's shapes; each line ends in a hash of the output, so two builds compare bit for bit.

    python tools/pconvt_micro.py                          # the in-tree library
    python tools/pconvt_micro.py --libs a.so,b.so,a.so    # builds interleaved, one process each
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


print("lib:", os.environ.get("DSGAN_HIP_LIB", "default"), flush=True)
tot = 0.0
N = 16
# (K input channels, M output channels, Hi input size, KS): the step's ConvTranspose forwards (KS 3)
# and PatchGAN stride-2 data-grads (KS 4)
for K, M, Hi, KS in [(128, 64, 128, 3), (256, 128, 64, 3), (1024, 512, 16, 3), (512, 256, 32, 3), (256, 128, 16, 3),
                     (128, 64, 64, 3), (128, 64, 32, 4), (64, 32, 64, 4)]:
    Ho = 2 * Hi
    g = torch.Generator(device="cuda").manual_seed(K + Hi)
    x = torch.randn(N, K, Hi, Hi, device="cuda", generator=g)
    wb = (torch.randn(KS * KS, M, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(M, device="cuda", generator=g)
    y = torch.empty(N, M, Ho, Ho, device="cuda")
    f = lambda: call("dsgan_pconvt", ptr(x), K * Hi * Hi, ptr(wb), ptr(b) if KS == 3 else None, ptr(y), M * Ho * Ho,
                     None, 0, N, K, M, Hi, Hi, Ho, Ho, KS, 2, 1, 0, 0.2, 0, stream())
    t = timeit(f)
    tot += t
    f()
    torch.cuda.synchronize()
    h = hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest()[:10]
    fl = 2.0 * N * Hi * Hi * 4 * M * K * (KS * KS / 4)
    print("K=%5d M=%4d Hi=%4d KS=%d | %7.1f us %6.0f TF/s | %s" % (K, M, Hi, KS, t, fl / t / 1e6, h), flush=True)
print("total: %.1f us" % tot, flush=True)
