"""Exact-fp32 pointwise GEMMs (csrc/pwf32.hip, v_mfma_f32_32x32x2_f32) vs float64 torch: the
MidMLKA 1x1 conv (DSGAN/models/model/MixConvNeXtML.py:85,112, fp32 by policy) and the fp32
parity mode's 1x1 convs.  f32 MFMA is exact f32 FMA arithmetic, so the bar is fp32 summation
order: 1e-6 relative."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup():
    import dsgan_hip
    from dsgan_hip import functional as HF
    dsgan_hip.require_gpu()
    return HF


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()


SHAPES = [(2, 128, 128, 32, 32), (3, 32, 32, 64, 64), (2, 256, 256, 16, 16), (1, 64, 96, 16, 24), (16, 128, 128, 8, 16),
          # the step's MidMLKA weight-grads (the 64 x 64 tile, the many-split plans)
          (16, 256, 256, 16, 16), (16, 128, 128, 32, 32), (4, 32, 32, 128, 128), (8, 64, 64, 64, 64)]


@pytest.mark.parametrize("shape", SHAPES)
def test_pwf32_fwd_dgrad_wgrad(shape):
    HF = _setup()
    N, Ci, Co, H, W = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(N, Ci, H, W, generator=g).cuda()
    w = (torch.randn(Co, Ci, 1, 1, generator=g) * 0.1).cuda()
    b = torch.randn(Co, generator=g).cuda()
    dy = torch.randn(N, Co, H, W, generator=g).cuda()
    xd, wd, bd, dyd = x.double(), w.double(), b.double(), dy.double()
    with HF.precision("fp32"):
        HF.IGEMM_TIMER.rec, HF.IGEMM_TIMER.on = [], True
        y = HF.conv_fwd_raw(x, w, b, 1, 0)
        dx = HF.conv_dgrad_raw(dy, w, tuple(x.shape), 1, 0)
        dw = torch.zeros_like(w)
        db = torch.full((Co,), 0.5, device="cuda")
        did_db = HF.conv_wgrad_raw(dy, x, dw, 1, 0, db=db)
        HF.IGEMM_TIMER.on = False
        fams = {r[4] for r in HF.IGEMM_TIMER.rec}
    torch.cuda.synchronize()
    if Ci > 36:   # (<= 36 input taps go to the exact VALU small_in kernel)
        assert fams == {"pwf32_kernel"}, fams
    yr = torch.nn.functional.conv2d(xd, wd, bd)
    dxr = torch.nn.functional.conv_transpose2d(dyd, wd)
    dwr = torch.einsum("nchw,nkhw->ck", dyd, xd).view(Co, Ci, 1, 1)
    assert rel(y, yr) < 1e-6 and rel(dx, dxr) < 1e-6 and rel(dw, dwr) < 1e-6, (rel(y, yr), rel(dx, dxr), rel(dw, dwr))
    if Ci > 36:   # the bias grad rides on the weight-grad's staged dy tiles (+= into db)
        assert did_db and rel(db, 0.5 + dyd.sum(dim=(0, 2, 3))) < 1e-6


def test_pwf32_epilogues_and_slices():
    """accumulate, the GELU act'-multiplier of the data-grad, and channel slices of a concat buffer
    (batch stride != C*H*W), through the C ABI directly."""
    HF = _setup()
    from dsgan_hip._lib import call, ptr, stream
    g = torch.Generator().manual_seed(1)
    N, Ci, Co, H, W = 2, 64, 128, 16, 16
    big = torch.randn(N, Ci + 32, H, W, generator=g).cuda()
    x = big[:, 32:]
    w = (torch.randn(Co, Ci, generator=g) * 0.1).cuda()
    y0 = torch.randn(N, Co, H, W, generator=g).cuda()
    y = y0.clone()
    call("dsgan_pw_gemm_f32", 0, ptr(w), 0, ptr(x), (Ci + 32) * H * W, ptr(y), Co * H * W, None, None, 0, Co,
         N * H * W, Ci, H * W, N, HF.ACT["gelu"], 0, 1, 0.2, None, 0, stream())
    pre = torch.einsum("kc,nchw->nkhw", w.double(), x.double())
    ref = y0.double() + torch.nn.functional.gelu(pre)
    gpre = torch.randn(N, Ci, H, W, generator=g).cuda()
    dy = torch.randn(N, Co, H, W, generator=g).cuda()
    dx = torch.empty(N, Ci, H, W, device="cuda")
    call("dsgan_pw_gemm_f32", 1, ptr(w), 0, ptr(dy), Co * H * W, ptr(dx), Ci * H * W, None, ptr(gpre), Ci * H * W,
         Ci, N * H * W, Co, H * W, N, 0, HF.ACT["gelu"], 0, 0.2, None, 0, stream())
    gp = gpre.double().requires_grad_(True)
    torch.nn.functional.gelu(gp).sum().backward()
    dref = torch.einsum("kc,nkhw->nchw", w.double(), dy.double()) * gp.grad
    torch.cuda.synchronize()
    assert rel(y, ref) < 1e-6 and rel(dx, dref) < 1e-5
