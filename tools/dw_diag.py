import sys, os
sys.path[:0] = ["/root/repo", "/root/repo/ds-gan_amd"]
import torch, torch.nn.functional as F
from dsgan_hip import functional as HF
import dsgan_hip
dsgan_hip.require_gpu()
torch.manual_seed(0)
for (N, C, H, K) in [(2, 8, 32, 3), (2, 8, 32, 5), (2, 8, 32, 7), (2, 8, 32, 9), (2, 3, 64, 7), (2, 64, 32, 7), (2, 128, 64, 7), (2, 256, 32, 7), (16, 16, 128, 7)]:
    x = torch.randn(N, C, H, H, dtype=torch.float64)
    w = torch.randn(C, 1, K, K, dtype=torch.float64) / K
    b = torch.randn(C, dtype=torch.float64)
    gy = torch.randn(N, C, H, H, dtype=torch.float64)
    y_ref = F.conv2d(x, w, b, padding=K // 2, groups=C)
    dx_ref = F.conv_transpose2d(gy, w, padding=K // 2, groups=C)
    xr = x.clone().requires_grad_(); wr = w.clone().requires_grad_()
    F.conv2d(xr, wr, None, padding=K // 2, groups=C).backward(gy)
    dw_ref = wr.grad
    xd, wd, bd, gd = (t.float().cuda() for t in (x, w, b, gy))
    y = HF.dwconv_raw(xd, wd, bd)
    dx = HF.dwconv_raw(gd, wd, None, flip=True)
    dw = torch.zeros_like(wd); db = torch.zeros_like(bd)
    HF._dw_wgrad(gd, xd, dw, db, K)
    r = lambda a, b_: ((a.double().cpu() - b_).norm() / b_.norm()).item()
    print(N, C, H, K, "y %.2e dx %.2e dw %.2e db %.2e" % (r(y, y_ref), r(dx, dx_ref), r(dw, dw_ref), r(db, gy.sum((0, 2, 3)))), flush=True)
