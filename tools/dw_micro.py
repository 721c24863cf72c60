"""Time the depthwise convs (dwconv.hip) at the DS-GAN step's shapes: the Block 7x7 forward, its
data-grad (flipped taps, accumulated into the shared input's grad), the weight-grad, and the MidMLKA
four-quarter forward.  Each line ends in a hash of the output bytes, so two builds can be compared
bit for bit.

    python tools/dw_micro.py                          # the in-tree library
    python tools/dw_micro.py --libs a.so,b.so,a.so    # builds interleaved, one process each
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


def digest(*ts):
    h = hashlib.sha1()
    for t in ts:
        t = t.detach().cpu()
        h.update((t.view(torch.int16) if t.dtype == torch.bfloat16 else t).numpy().tobytes())
    return h.hexdigest()[:10]


print("lib:", os.environ.get("DSGAN_HIP_LIB", "default"), flush=True)
tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
for N, C, H in [(16, 128, 256), (16, 256, 128), (16, 512, 64), (16, 1024, 32), (16, 64, 128), (16, 128, 64),
                (16, 256, 32), (16, 3, 256)]:
    K, HW = 7, H * H
    g = torch.Generator(device="cuda").manual_seed(C + H)
    x = torch.randn(N, C, H, H, device="cuda", generator=g)
    dy = torch.randn(N, C, H, H, device="cuda", generator=g)
    w = torch.randn(C, 1, K, K, device="cuda", generator=g) * 0.1
    b = torch.randn(C, device="cuda", generator=g)
    y = torch.empty_like(x)
    dx0 = torch.randn(N, C, H, H, device="cuda", generator=g)
    dx = dx0.clone()
    dw = torch.zeros(C, 1, K, K, device="cuda")
    db = torch.zeros(C, device="cuda")
    ws = torch.empty(max(1, L.dsgan_dwconv_wgrad_workspace(N, C, H, H, K, 1)), device="cuda")
    fwd = lambda: call("dsgan_dwconv_fwd", ptr(x), C * HW, ptr(w), ptr(b), ptr(y), C * HW, N, C, H, H, K, 0, 0, stream())
    dgr = lambda: call("dsgan_dwconv_fwd", ptr(dy), C * HW, ptr(w), None, ptr(dx), C * HW, N, C, H, H, K, 1, 1,
                       stream())
    wgr = lambda: call("dsgan_dwconv_wgrad", ptr(dy), C * HW, ptr(x), C * HW, ptr(dw), ptr(db), N, C, H, H, K,
                       ptr(ws), ws.numel(), stream())
    t = [timeit(fwd), timeit(dgr), timeit(wgr)]
    for k, v in zip(("fwd", "dgrad", "wgrad"), t):
        tot[k] += v
    # one clean pass of each for the digest
    fwd()
    dx.copy_(dx0)
    dgr()
    wgr()
    torch.cuda.synchronize()
    print("C=%4d H=%3d | fwd %7.1f  dgrad %7.1f  wgrad %7.1f us | %s" % (C, H, *t, digest(y, dx, dw, db)), flush=True)
for N, C, H in [(16, 128, 128), (16, 32, 128), (16, 128, 64), (16, 64, 64), (16, 128, 32)]:
    q, HW = C // 4, H * H
    torch.manual_seed(C + H)
    x = torch.randn(N, C, H, H, device="cuda")
    wq = [torch.randn(q, 1, k, k, device="cuda") * 0.1 for k in (3, 5, 7, 9)]
    bq = [torch.randn(q, device="cuda") for _ in range(4)]
    y = torch.empty_like(x)
    f = lambda: call("dsgan_dwconv_multi_fwd", ptr(x), C * HW, ptr(wq[0]), ptr(bq[0]), ptr(wq[1]), ptr(bq[1]),
                     ptr(wq[2]), ptr(bq[2]), ptr(wq[3]), ptr(bq[3]), ptr(y), C * HW, N, q, H, H, 0, 0, stream())
    dy = torch.randn(N, C, H, H, device="cuda")
    gw = [torch.zeros(q, 1, k, k, device="cuda") for k in (3, 5, 7, 9)]
    gb = [torch.zeros(q, device="cuda") for _ in range(4)]
    wsp = torch.empty(max(1, L.dsgan_dwconv_multi_wgrad_workspace(N, q, H, H)), device="cuda")
    fw = lambda: call("dsgan_dwconv_multi_wgrad", ptr(dy), C * HW, ptr(x), C * HW, ptr(gw[0]), ptr(gb[0]), ptr(gw[1]),
                      ptr(gb[1]), ptr(gw[2]), ptr(gb[2]), ptr(gw[3]), ptr(gb[3]), N, q, H, H, ptr(wsp), wsp.numel(),
                      stream())
    t, tw = timeit(f), timeit(fw)
    tot["fwd"] += t
    tot["wgrad"] += tw
    f()
    fw()
    torch.cuda.synchronize()
    print("multi C=%4d H=%3d | fwd %7.1f  wgrad %7.1f us | %s" % (C, H, t, tw, digest(y, *gw, *gb)), flush=True)
print("totals: " + "  ".join("%s %.1f us" % kv for kv in tot.items()), flush=True)
