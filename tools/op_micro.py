"""Time one contraction at a DS-GAN shape (for rocprofv3 counter passes).
usage: op_micro.py {convt|dgrad4|vgg3|wgrad3} [iters]"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
import dsgan_hip
from dsgan_hip import functional as HF
dsgan_hip.require_gpu()
HF.set_precision("bf16")
which = sys.argv[1] if len(sys.argv) > 1 else "convt"
it = int(sys.argv[2]) if len(sys.argv) > 2 else 20
N = 16
if which == "convt":      # u4: ConvT 128@128^2 -> 64@256^2
    x = torch.randn(N, 128, 128, 128, device="cuda"); w = torch.randn(128, 64, 3, 3, device="cuda") * 0.03
    b = torch.randn(64, device="cuda")
    f = lambda: HF.conv_dgrad_raw(x, w, (N, 64, 256, 256), 2, 1, bias=b)
    fl = 2.0 * N * 64 * 128 * 9 * 128 * 128
elif which == "vgg3":     # conv1_2 64->64 at 256^2
    x = torch.randn(N, 64, 256, 256, device="cuda"); w = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    b = torch.randn(64, device="cuda")
    f = lambda: HF.conv_fwd_raw(x, w, b, 1, 1, act="relu")
    fl = 2.0 * N * 64 * 64 * 9 * 256 * 256
elif which == "pwfwd":     # uc1 pwconv2: gelu(z) 4096 -> 512 at 32^2
    x = torch.randn(N, 4096, 32, 32, device="cuda"); w = torch.randn(512, 4096, 1, 1, device="cuda") * 0.02
    y = torch.empty(N, 512, 32, 32, device="cuda")
    f = lambda: HF.conv_fwd_raw(x, w, None, 1, 0, out=y, xact="gelu")
    fl = 2.0 * N * 512 * 4096 * 1024
elif which == "pwfwd2":    # uc2 pwconv1: 512 -> 2048 at 64^2
    x = torch.randn(N, 512, 64, 64, device="cuda"); w = torch.randn(2048, 512, 1, 1, device="cuda") * 0.02
    b = torch.randn(2048, device="cuda")
    f = lambda: HF.conv_fwd_raw(x, w, b, 1, 0)
    fl = 2.0 * N * 2048 * 512 * 4096
elif which == "pwdgrad":   # uc2 pwconv2 data-grad: 256 -> 2048 at 64^2 (* gelu'(z))
    dy = torch.randn(N, 256, 64, 64, device="cuda"); w = torch.randn(256, 2048, 1, 1, device="cuda") * 0.02
    z = torch.randn(N, 2048, 64, 64, device="cuda")
    f = lambda: HF.conv_dgrad_raw(dy, w, (N, 2048, 64, 64), 1, 0, gpre=z, gact="gelu")
    fl = 2.0 * N * 2048 * 256 * 4096
elif which == "pwwgrad":   # uc2 pwconv1 weight-grad: dz 2048 x h 512 over 16*64^2 pixels
    dz = torch.randn(N, 2048, 64, 64, device="cuda"); x = torch.randn(N, 512, 64, 64, device="cuda")
    dw = torch.zeros(2048, 512, 1, 1, device="cuda")
    f = lambda: HF.conv_wgrad_raw(dz, x, dw, 1, 0)
    fl = 2.0 * N * 2048 * 512 * 4096
else:
    raise SystemExit("unknown op")
f(); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(it):
    f()
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / it
print("%s: %.3f ms  %.1f TF/s" % (which, ms, fl / ms / 1e9), flush=True)
