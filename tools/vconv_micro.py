"""In-process A/B of the VGG16 3x3 conv kernels (vggconv.hip) at the step's shapes (batch 16, 256^2
input): the LDS-DMA ring kernel (dsgan_vconv_tune(0, 0)) vs the register-staged one (1), and the ring with
kw-major taps (3: another fp32 summation order, compared by relative error).  Outputs of
the two forms must be bitwise equal (same operands, same per-output accumulation order).

    python tools/vconv_micro.py [--it 20]
    python tools/vconv_micro.py --libs a.so,b.so,a.so [--it 20]   # builds interleaved, one process each
"""
import argparse
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2 and sys.argv[1] == "--libs":
    # A/B of builds: one child process per listed library, in order (this parent never touches the GPU)
    rc = 0
    for lib_path in sys.argv[2].split(","):
        env = dict(os.environ, DSGAN_HIP_LIB=os.path.join(REPO, lib_path))
        rc |= subprocess.run([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[3:], env=env).returncode
    sys.exit(rc)
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch  # noqa: E402
import dsgan_hip  # noqa: E402
from dsgan_hip import _lib  # noqa: E402
from dsgan_hip._lib import call, ptr, stream  # noqa: E402

N = 16
# the three kernel forms compared (dsgan_vconv_tune key 0); VCONV_MODES="3,4,5" compares the ring variants
MODES = tuple(int(m) for m in os.environ.get("VCONV_MODES", "1,0,3").split(","))
# (name, K in, M out, H, dgrad): the forward convs of vgg.py:15-24 and the data-grads of the backward walk
LAYERS = [("c1_2", 64, 64, 256, 0), ("c2_1", 64, 128, 128, 0), ("c2_2", 128, 128, 128, 0), ("c3_1", 128, 256, 64, 0),
          ("c3_2", 256, 256, 64, 0), ("c4_1", 256, 512, 32, 0), ("c4_2", 512, 512, 32, 0),
          ("d1_2", 64, 64, 256, 1), ("d2_1", 128, 64, 128, 1), ("d2_2", 128, 128, 128, 1), ("d3_1", 256, 128, 64, 1),
          ("d3_2", 256, 256, 64, 1), ("d4_1", 512, 256, 32, 1), ("d4_2", 512, 512, 32, 1)]


def timeit(fn, it):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(it):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--it", type=int, default=20)
    a = ap.parse_args()
    dsgan_hip.require_gpu()
    lib = _lib.load()
    old = lib.dsgan_vconv_tune(0, -1)
    g = torch.Generator(device="cuda").manual_seed(0)
    tot = [0.0, 0.0, 0.0]
    print("%-6s %5s %5s %4s | %9s %9s %9s | %7s %7s %7s | bitwise | kwm rel" % (
        "layer", "K", "M", "H", "old us", "dma us", "kwm us", "old TF", "dma TF", "kwm TF"))
    for name, K, M, H, dgrad in LAYERS:
        Co, Ci = (K, M) if dgrad else (M, K)
        W = torch.randn(Co, Ci, 3, 3, device="cuda", generator=g) * 0.05
        Wt = torch.empty(9 * Co * Ci, device="cuda", dtype=torch.bfloat16)
        call("dsgan_vconv_wtrans", ptr(W), ptr(Wt), Co, Ci, dgrad, stream())
        X = torch.randn(N * K * H * H, device="cuda", generator=g).to(torch.bfloat16)
        bias = None if dgrad else torch.randn(M, device="cuda", generator=g)
        mask = torch.randn(N * M * H * H, device="cuda", generator=g).to(torch.bfloat16) if dgrad else None
        ys = []
        ts = []
        for mode in MODES:
            lib.dsgan_vconv_tune(0, mode)
            Y = torch.empty(N * M * H * H, device="cuda", dtype=torch.bfloat16)
            fn = lambda Y=Y: call("dsgan_vconv3x3", ptr(X), ptr(Wt), ptr(bias), ptr(mask), ptr(Y), 0, 0 if dgrad else 1,
                                  N, K, M, H, H, stream())
            fn()
            torch.cuda.synchronize()
            ys.append(Y.clone())
            ts.append(timeit(fn, a.it))
        fl = 2.0 * N * M * K * 9 * H * H
        same = torch.equal(ys[0], ys[1])
        d = (ys[2].float() - ys[0].float()).norm() / ys[0].float().norm().clamp_min(1e-30)
        for q in range(3):
            tot[q] += ts[q]
        print("%-6s %5d %5d %4d | %9.1f %9.1f %9.1f | %7.1f %7.1f %7.1f | %s | %.2e" % (
            name, K, M, H, ts[0], ts[1], ts[2], fl / ts[0] / 1e6, fl / ts[1] / 1e6, fl / ts[2] / 1e6, same, d.item()),
            flush=True)
    lib.dsgan_vconv_tune(0, old)
    print("total: old %.1f us, dma %.1f us, kwm %.1f us" % tuple(tot))


if __name__ == "__main__":
    main()
