"""Time the fused MLP kernels (mlp.hip) at the DS-GAN block shapes, as the training step calls them
(bf16 h from the block's InstanceNorm): forward, backward dh-only + weight-grad kernel, and the
backward with bf16 g / dz written for the pwgemm weight-grads.

    python tools/mlp_micro.py            # DSGAN_HIP_LIB=<other .so> to time another build
    python tools/mlp_micro.py --libs a.so,b.so,a.so   # builds interleaved, one process each
"""
import os, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2 and sys.argv[1] == "--libs":
    # A/B of builds: one child process per listed library, in order (this parent never touches the GPU)
    rc = 0
    for lib_path in sys.argv[2].split(","):
        env = dict(os.environ, DSGAN_HIP_LIB=os.path.join(REPO, lib_path))
        rc |= subprocess.run([sys.executable, "-u", os.path.abspath(__file__)], env=env).returncode
    sys.exit(rc)
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
from dsgan_hip._lib import call, ptr, stream
import dsgan_hip

dsgan_hip.require_gpu()
N = 16
SHAPES = [("uc4", 128, 64, 256), ("uc3", 256, 128, 128), ("c2", 64, 128, 128), ("c3", 128, 256, 64)]
if os.environ.get("MLP_SHAPES"):
    SHAPES = [s for s in SHAPES if s[0] in os.environ["MLP_SHAPES"].split(",")]


def timeit(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


lib = dsgan_hip._lib.load()
print("lib:", os.environ.get("DSGAN_HIP_LIB", "default"), flush=True)
for name, C, P, H in SHAPES:
    HW = H * H
    C4 = 4 * C
    torch.manual_seed(0)
    h = torch.randn(N, C, H, H, device="cuda").bfloat16()
    dy = torch.randn(N, P, H, H, device="cuda")
    out = torch.zeros(N, P, H, H, device="cuda")
    w1 = (torch.randn(C4, C, device="cuda") / C ** 0.5).bfloat16()
    w2 = (torch.randn(P, C4, device="cuda") / C4 ** 0.5).bfloat16()
    b1 = torch.randn(C4, device="cuda") * 0.1
    b2 = torch.randn(P, device="cuda") * 0.1
    g = torch.empty(N, C4, H, H, device="cuda", dtype=torch.bfloat16)
    dz = torch.empty_like(g)
    dh = torch.empty(N, C, H, H, device="cuda")
    gw1, gb1, gw2 = torch.zeros(C4, C, device="cuda"), torch.zeros(C4, device="cuda"), torch.zeros(P, C4, device="cuda")
    wsp = torch.empty(lib.dsgan_mlp_wgrad_workspace(C, P, HW, N), device="cuda")
    f = lambda: call("dsgan_mlp_fwd", ptr(h), C * HW, 1, ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(out), P * HW, N, C, P,
                     HW, 1, stream())
    bd = lambda: call("dsgan_mlp_bwd", ptr(h), C * HW, 1, ptr(dy), P * HW, ptr(w1), ptr(b1), ptr(w2), ptr(dh), C * HW,
                      None, None, None, N, C, P, HW, stream())
    wg = lambda: call("dsgan_mlp_wgrad", ptr(h), C * HW, 1, ptr(dy), P * HW, ptr(w1), ptr(b1), ptr(w2), ptr(gw1),
                      ptr(gb1), ptr(gw2), ptr(wsp), wsp.numel(), N, C, P, HW, stream())
    bg = lambda: call("dsgan_mlp_bwd", ptr(h), C * HW, 1, ptr(dy), P * HW, ptr(w1), ptr(b1), ptr(w2), ptr(dh), C * HW,
                      ptr(g), ptr(dz), None, N, C, P, HW, stream())
    tf, tbd, twg, tbg = timeit(f), timeit(bd), timeit(wg), timeit(bg)
    # checksums so that two builds can be compared for identical results
    f(); bd(); wg(); torch.cuda.synchronize()
    cs = (out.double().sum().item(), dh.double().sum().item(), gw1.double().abs().sum().item(),
          gw2.double().abs().sum().item(), gb1.double().abs().sum().item())
    # knob A/B of the backward with g / dz out (dsgan_mlp_tune key 0: 0 LDS-DMA ring, 1 register-staged,
    # 2 the ring with precomputed addresses)
    ab = ""
    if C == 256:
        old = lib.dsgan_mlp_tune(0, -1)
        res = {}
        for mode in (1, 0, 2):
            lib.dsgan_mlp_tune(0, mode)
            t = timeit(bg)
            bg(); torch.cuda.synchronize()
            res[mode] = (t, dh.clone(), g.clone(), dz.clone())
        lib.dsgan_mlp_tune(0, old)
        same = [all(torch.equal(a, b) for a, b in zip(res[m][1:], res[1][1:])) for m in (0, 2)]
        ab = " | bwd-g/dz staged %.3f dma %.3f (bitwise %s) dma-addr %.3f ms (bitwise %s)" % (
            res[1][0], res[0][0], same[0], res[2][0], same[1])
    fl = 2.0 * N * HW * (C4 * C + C4 * P)
    print("%-4s C=%4d P=%4d HW=%6d | fwd %.3f ms (%.0f TF/s) | bwd-dh %.3f | wgrad %.3f | bwd-g/dz %.3f ms | cs %s%s"
          % (name, C, P, HW, tf, fl / tf / 1e9, tbd, twg, tbg, " ".join("%.6e" % c for c in cs), ab), flush=True)
    del h, dy, out, g, dz, dh, wsp
