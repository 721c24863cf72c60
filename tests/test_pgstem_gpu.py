"""PatchGAN stem kernels (csrc/pgstem.hip): NLayerDiscriminator layer 0 = Conv2d(input_nc, ndf, 4,
stride 2, pad 1) + bias + LeakyReLU(0.2, True) (DSGAN/models/networks.py:543-545), forward and
backward, against the float64 torch CPU op (what the reference runs, in double) and against the
generic conv path it replaces (HF.PGSTEM off: implicit GEMM + LeakyReLU backward + channel sum).

Every product in the stem is exact fp32 in both precision modes, so the bar is the fp32
accumulation bar (rel-l2 1e-5 vs float64) in bf16 mode too.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    import dsgan_hip
    dsgan_hip.require_gpu()
    yield
    dsgan_hip.set_precision("fp32")
    from dsgan_hip import functional as HF
    HF.PGSTEM[0] = True


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()


def _ref(x, w, b, dy):
    xd, wd, bd = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    y = F.leaky_relu(F.conv2d(xd, wd, bd, stride=2, padding=1), 0.2)
    y.backward(dy.double())
    return y.detach(), xd.grad, wd.grad, bd.grad


def _run(x, w, b, dy, prec="fp32", stem=True, need_x=True):
    from dsgan_hip import functional as HF
    HF.set_precision(prec)
    HF.PGSTEM[0] = stem
    xg = x.to(DEV).requires_grad_(need_x)
    wp = torch.nn.Parameter(w.to(DEV))
    bp = torch.nn.Parameter(b.to(DEV))
    wp.grad = torch.zeros_like(wp)
    bp.grad = torch.zeros_like(bp)
    y = HF.conv2d(xg, wp, bp, stride=2, pad=1, act="lrelu")
    assert (type(y.grad_fn).__name__ == "PatchStemFnBackward") == stem
    y.backward(dy.to(DEV))
    torch.cuda.synchronize()
    HF.PGSTEM[0] = True
    return y.detach(), (xg.grad if need_x else None), wp.grad, bp.grad


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("N,Cin,Cout,H,W", [(2, 6, 32, 256, 256), (3, 6, 32, 64, 64), (1, 3, 64, 128, 128),
                                            (2, 6, 64, 64, 192), (1, 6, 32, 512, 512)])
def test_stem_vs_float64(prec, N, Cin, Cout, H, W):
    from dsgan_hip import _lib
    assert _lib.load().dsgan_pgstem_supported(Cin, Cout, H, W)
    g = torch.Generator().manual_seed(N * 100 + Cin * 10 + H)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 4, 4, generator=g) * 0.1
    b = torch.randn(Cout, generator=g) * 0.1
    dy = torch.randn(N, Cout, H // 2, W // 2, generator=g)
    y, dx, dw, db = _run(x, w, b, dy, prec)
    ry, rdx, rdw, rdb = _ref(x, w, b, dy)
    assert rel(y, ry) < 1e-6
    assert rel(dx, rdx) < 1e-6
    assert rel(dw, rdw) < 1e-5
    assert rel(db, rdb) < 1e-5


@pytest.mark.parametrize("Cin,Cout,H,W", [(6, 32, 128, 128), (6, 32, 256, 256), (3, 64, 64, 192)])
def test_stem_matches_generic_path_fp32(Cin, Cout, H, W):
    """Same layer through the generic conv path (fp32 mode: exact f32 MFMA).  The forward is the
    same fp32 fma chain, so y is bit-identical (a near-zero pre-activation is a LeakyReLU kink
    downstream: the stem must not move it); the gradients agree to the fp32 accumulation bar."""
    g = torch.Generator().manual_seed(7 + H)
    x = torch.randn(2, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 4, 4, generator=g) * 0.05
    b = torch.randn(Cout, generator=g) * 0.05
    dy = torch.randn(2, Cout, H // 2, W // 2, generator=g)
    a = _run(x, w, b, dy, "fp32", stem=True)
    r = _run(x, w, b, dy, "fp32", stem=False)
    assert torch.equal(a[0], r[0])
    for u, v in zip(a[1:], r[1:]):
        assert rel(u, v) < 2e-6


def test_stem_deterministic_and_frozen_paths():
    """Two identical backward passes give the same bits; x without grad skips the data-grad; a
    frozen weight (the G step's D pass) leaves the parameters untouched and still returns dx."""
    from dsgan_hip import functional as HF
    HF.set_precision("bf16")
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 6, 256, 256, generator=g)
    w = torch.randn(32, 6, 4, 4, generator=g) * 0.05
    b = torch.randn(32, generator=g) * 0.05
    dy = torch.randn(2, 32, 128, 128, generator=g)
    r1 = _run(x, w, b, dy, "bf16", need_x=False)
    r2 = _run(x, w, b, dy, "bf16", need_x=False)
    assert r1[1] is None
    for u, v in zip(r1, r2):
        if u is not None:
            assert torch.equal(u, v)
    wp = torch.nn.Parameter(w.to(DEV), requires_grad=False)
    bp = torch.nn.Parameter(b.to(DEV), requires_grad=False)
    xg = x.to(DEV).requires_grad_(True)
    y = HF.conv2d(xg, wp, bp, stride=2, pad=1, act="lrelu")
    y.backward(dy.to(DEV))
    assert wp.grad is None and bp.grad is None
    _, rdx, _, _ = _ref(x, w, b, dy)
    assert rel(xg.grad, rdx) < 1e-6


def test_stem_dgrad_accumulates_into_slices():
    """dgrad accumulate=1 into a channel slice of a bigger buffer (the box / concat path), read
    through the C ABI directly."""
    from dsgan_hip import _lib
    from dsgan_hip._lib import call, ptr, stream
    g = torch.Generator().manual_seed(3)
    N, Cin, Cout, H, W = 2, 6, 32, 64, 128
    w = torch.randn(Cout, Cin, 4, 4, generator=g) * 0.1
    y = torch.randn(N, Cout, H // 2, W // 2, generator=g)
    dy = torch.randn(N, Cout, H // 2, W // 2, generator=g)
    big0 = torch.randn(N, Cin + 2, H, W, generator=g)
    big = big0.to(DEV)
    dst = big[:, 2:]
    dyd, yd, wd = dy.to(DEV), y.to(DEV), w.to(DEV)   # held: a temporary's block is reused at once
    call("dsgan_pgstem_dgrad", ptr(dyd), dy[0].numel(), ptr(yd), y[0].numel(), ptr(wd), ptr(dst), big[0].numel(),
         N, Cin, Cout, H, W, 0.2, 1, stream())
    torch.cuda.synchronize()
    dyp = torch.where(y > 0, dy, dy * 0.2).double()
    ref = big0.double().clone()
    ref[:, 2:] += torch.nn.grad.conv2d_input((N, Cin, H, W), w.double(), dyp, stride=2, padding=1)
    assert rel(big, ref) < 1e-6
    assert not _lib.load().dsgan_pgstem_supported(6, 32, 60, 64)
    assert not _lib.load().dsgan_pgstem_supported(6, 48, 64, 64)


# ---- PatchGAN head (csrc/pglast.hip): Conv2d(ndf * 8, 1, 4, stride 1, pad 1), networks.py:567-568 ----

@pytest.mark.parametrize("N,K,H,W", [(16, 256, 31, 31), (2, 256, 63, 63), (3, 64, 7, 9), (2, 40, 15, 15)])
def test_head_vs_float64(N, K, H, W):
    from dsgan_hip import _lib
    from dsgan_hip import functional as HF
    assert _lib.load().dsgan_pglast_supported(K, H, W)
    HF.set_precision("bf16")
    g = torch.Generator().manual_seed(N * 1000 + K + H)
    x = torch.randn(N, K, H, W, generator=g)
    w = torch.randn(1, K, 4, 4, generator=g) * 0.05
    b = torch.randn(1, generator=g)
    dy = torch.randn(N, 1, H - 1, W - 1, generator=g)
    xg = x.to(DEV).requires_grad_(True)
    wp = torch.nn.Parameter(w.to(DEV))
    bp = torch.nn.Parameter(b.to(DEV))
    wp.grad = torch.zeros_like(wp)
    bp.grad = torch.zeros_like(bp)
    y = HF.conv2d(xg, wp, bp, stride=1, pad=1)
    y.backward(dy.to(DEV))
    torch.cuda.synchronize()
    xd, wd, bd = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = F.conv2d(xd, wd, bd, stride=1, padding=1)
    yr.backward(dy.double())
    assert rel(y, yr) < 1e-6
    assert rel(xg.grad, xd.grad) < 1e-6
    assert rel(wp.grad, wd.grad) < 1e-5
    assert rel(bp.grad, bd.grad) < 1e-6


def test_head_matches_generic_path_and_is_deterministic():
    """Same layer with HF.PGLAST off (small_out / implicit GEMM / wgrad_small): equal to the fp32
    bar; two runs of the head kernels give the same bits."""
    from dsgan_hip import functional as HF
    HF.set_precision("fp32")
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 256, 31, 31, generator=g)
    w = torch.randn(1, 256, 4, 4, generator=g) * 0.05
    b = torch.randn(1, generator=g)
    dy = torch.randn(4, 1, 30, 30, generator=g)
    res = []
    for on in (True, True, False):
        HF.PGLAST[0] = on
        xg = x.to(DEV).requires_grad_(True)
        wp = torch.nn.Parameter(w.to(DEV))
        bp = torch.nn.Parameter(b.to(DEV))
        wp.grad = torch.zeros_like(wp)
        bp.grad = torch.zeros_like(bp)
        y = HF.conv2d(xg, wp, bp, stride=1, pad=1)
        y.backward(dy.to(DEV))
        torch.cuda.synchronize()
        res.append((y.detach(), xg.grad, wp.grad, bp.grad))
    HF.PGLAST[0] = True
    for u, v, r in zip(res[0], res[1], res[2]):
        assert torch.equal(u, v)
        assert rel(u, r) < 2e-6
