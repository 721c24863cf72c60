"""Per-kernel parity: every HIP op (through the C-ABI) vs the same op on PyTorch-CPU fp32/fp64,
i.e. the exact CPU math the reference runs (DSGAN's modules are torch ops).

fp32 mode (exact f32 MFMA) must match to ~1e-5 relative; bf16 mode (bf16 operands, fp32
accumulation) to the bf16 rounding bar stated per test.  Index tensors are bit-exact.
"""
import math

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


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()


def _leaf(t):
    return t.detach().clone().to(DEV).requires_grad_(True)


def _param(t):
    p = torch.nn.Parameter(t.detach().clone().to(DEV))
    p.grad = torch.zeros_like(p)
    return p


TOL = {"fp32": 2e-5, "bf16": 1.5e-2, "fp16": 3e-3}   # fp16: 3 more mantissa bits than bf16
HALVES = ["bf16", "fp16"]


def _hdt(half):
    return torch.float16 if half == "fp16" else torch.bfloat16


def _ulp(half):
    """relative rounding bound of one RNE conversion to the 16-bit type"""
    return 2.0 ** -11 if half == "fp16" else 2.0 ** -8


def _q(t, prec):
    """16-bit modes round MFMA operands to bf16 / fp16: the reference sees the same rounded
    operands, so activation masks agree and the bar measures accumulation/rounding only."""
    return t.to(_hdt(prec)).float() if prec in HALVES else t


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("N,Cin,H,W,Cout,K,s,p", [
    (2, 3, 16, 16, 12, 1, 1, 0),       # c1.pwconv1 shape class (K tiny)
    (2, 64, 16, 16, 256, 1, 1, 0),
    (3, 130, 9, 7, 70, 1, 1, 0),       # ragged M/N/K tails
    (2, 3, 20, 20, 64, 3, 1, 1),       # VGG conv1_1 (K=27)
    (2, 64, 18, 18, 128, 3, 1, 1),
    (2, 64, 16, 16, 3, 3, 1, 1),       # G head 64->3
    (2, 6, 32, 32, 32, 4, 2, 1),       # PatchGAN layer 0
    (2, 64, 16, 16, 128, 4, 2, 1),
    (2, 128, 9, 9, 256, 4, 1, 1),      # PatchGAN s1 layers
    (2, 256, 8, 8, 1, 4, 1, 1),
    (3, 64, 40, 36, 3, 3, 1, 1),       # skinny direct kernels at larger planes
    (4, 256, 31, 31, 1, 4, 1, 1),      # PatchGAN last layer shape (K-split atomics)
    (2, 3, 64, 64, 32, 1, 1, 0),       # to32 (wgrad with Cin = 3)
    (2, 12, 64, 64, 64, 1, 1, 0),      # c1 pwconv2-like: data-grad 64 -> 12 (pw_small, 4-channel load steps)
    (2, 12, 32, 32, 70, 1, 1, 0),      # ... with a channel remainder after the load steps
    (2, 6, 66, 66, 64, 4, 2, 1),       # PatchGAN layer 0 (stride-2 data-grad into 6 channels)
    (2, 1024, 96, 96, 1024, 1, 1, 0),  # wide, deep 1x1 fwd + data-grad: 256-row M tiles (K >= 1024)
    (2, 64, 8, 256, 3, 3, 1, 1),       # G head at full width: thin3.hip row strips (act=None)
    (1, 33, 12, 512, 4, 3, 1, 1),      # thin3: two 256-column segments per row, M = 4, odd K
    (2, 9, 4, 256, 1, 3, 1, 1),        # thin3: M = 1
])
def test_conv2d(prec, N, Cin, H, W, Cout, K, s, p):
    from dsgan_hip import functional as HF
    if prec == "fp32" and Cin * Cout >= 256 * 1024:
        pytest.skip("wide 1x1 shapes target the bf16 pwgemm 256-row tiles (fp32 mode runs igemm)")
    HF.set_precision(prec)
    g = torch.Generator().manual_seed(N * 1000 + Cin + Cout + K)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, K, K, generator=g) / math.sqrt(Cin * K * K)
    b = torch.randn(Cout, generator=g) * 0.1
    x, w = _q(x, prec), _q(w, prec)
    for act in (None, "lrelu", "relu"):
        xr, wr, br = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
        y_ref = F.conv2d(xr, wr, br, stride=s, padding=p)
        if act == "lrelu":
            y_ref = F.leaky_relu(y_ref, 0.2)
        elif act == "relu":
            y_ref = F.relu(y_ref)
        gy = torch.randn(y_ref.shape, generator=g)
        y_ref.backward(gy)
        xd, wd, bd = _leaf(x), _param(w), _param(b)
        y = HF.conv2d(xd, wd, bd, stride=s, pad=p, act=act)
        y.backward(gy.to(DEV))
        torch.cuda.synchronize()
        tol = TOL[prec]
        assert rel(y, y_ref) < tol, ("fwd", act)
        assert rel(xd.grad, xr.grad) < tol * 2, ("dgrad", act)
        assert rel(wd.grad, wr.grad) < tol * 2, ("wgrad", act)
        assert rel(bd.grad, br.grad) < max(1e-5, tol), ("bgrad", act)


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("N,Ci,Co,H", [(2, 64, 32, 8), (2, 128, 64, 5), (1, 256, 128, 16),
                                       (2, 1024, 512, 16)])   # u1 shape: split-K tconv data-grad
def test_conv_transpose(prec, N, Ci, Co, H):
    from dsgan_hip import functional as HF
    HF.set_precision(prec)
    g = torch.Generator().manual_seed(Ci + Co + H)
    x = _q(torch.randn(N, Ci, H, H + 1, generator=g), prec)
    w = _q(torch.randn(Ci, Co, 3, 3, generator=g) / math.sqrt(Ci * 9), prec)
    b = torch.randn(Co, generator=g) * 0.1
    xr, wr, br = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    y_ref = F.conv_transpose2d(xr, wr, br, stride=2, padding=1, output_padding=1)
    gy = torch.randn(y_ref.shape, generator=g)
    y_ref.backward(gy)
    xd, wd, bd = _leaf(x), _param(w), _param(b)
    y = HF.conv_transpose3s2(xd, wd, bd)
    y.backward(gy.to(DEV))
    tol = TOL[prec]
    assert y.shape == y_ref.shape
    assert rel(y, y_ref) < tol
    assert rel(xd.grad, xr.grad) < 2 * tol
    assert rel(wd.grad, wr.grad) < 2 * tol
    assert rel(bd.grad, br.grad) < 1e-5


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("N,C,H,P", [(2, 3, 16, 64), (2, 64, 8, 128), (2, 128, 12, 64),
                                     (2, 256, 16, 512),    # unfused large block: bf16 g = gelu(z) path
                                     (2, 256, 96, 1024)])  # 4C = 1024 = K of the data-grad: 256-row M tiles
def test_pw_mlp(prec, N, C, H, P):
    """Block tail: shortcut(x) + W2 gelu(W1 h + b1) + b2 (MixConvNeXtML.py:236-242)."""
    from dsgan_hip import functional as HF
    HF.set_precision(prec)
    g = torch.Generator().manual_seed(C + P)
    h = _q(torch.randn(N, C, H, H, generator=g), prec)
    x = _q(torch.randn(N, C, H, H, generator=g), prec)
    w1 = _q(torch.randn(4 * C, C, generator=g) / math.sqrt(C), prec)
    b1 = torch.randn(4 * C, generator=g) * 0.1
    w2 = _q(torch.randn(P, 4 * C, generator=g) / math.sqrt(4 * C), prec)
    b2 = torch.randn(P, generator=g) * 0.1
    ws = _q(torch.randn(P, C, 1, 1, generator=g) / math.sqrt(C), prec)
    R = [t.clone().requires_grad_() for t in (h, x, w1, b1, w2, b2, ws)]
    t = F.linear(R[0].permute(0, 2, 3, 1), R[2], R[3])
    t = F.linear(F.gelu(t), R[4], R[5]).permute(0, 3, 1, 2)
    y_ref = F.conv2d(R[1], R[6]) + t
    gy = torch.randn(y_ref.shape, generator=g)
    y_ref.backward(gy)
    hd, xd = _leaf(h), _leaf(x)
    P_ = [_param(t) for t in (w1, b1, w2, b2, ws)]
    y = HF.pw_mlp(hd, xd, *P_)
    y.backward(gy.to(DEV))
    tol = TOL[prec]
    assert rel(y, y_ref) < tol
    assert rel(hd.grad, R[0].grad) < 2 * tol
    assert rel(xd.grad, R[1].grad) < 2 * tol
    for pd, pr in zip(P_, R[2:]):
        assert rel(pd.grad, pr.grad) < 2 * tol


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("N,C,H,P", [(2, 64, 16, 128),     # fused MLP kernels (mlp.hip)
                                     (2, 256, 16, 512),    # unfused bf16 g / gp / dz path
                                     (2, 3, 16, 64)])      # fp32-z path (tiny block)
def test_block_tail_norm(prec, N, C, H, P):
    """pw_mlp(norm=True): the block's InstanceNorm folded into the MLP node (bf16 h in bf16 mode)
    vs a torch fp32 reference of IN -> Linear -> GELU -> Linear (+ shortcut), and BITWISE equal to
    the unfolded pair instance_norm(d) -> pw_mlp(h): storing h in bf16 changes no bit because its
    only readers round it to bf16 on load."""
    from dsgan_hip import functional as HF
    HF.set_precision(prec)
    g = torch.Generator().manual_seed(3 * C + P)
    d = torch.randn(N, C, H, H, generator=g) * 2 + 0.5
    x = _q(torch.randn(N, C, H, H, generator=g), prec)
    w1 = _q(torch.randn(4 * C, C, generator=g) / math.sqrt(C), prec)
    b1 = torch.randn(4 * C, generator=g) * 0.1
    w2 = _q(torch.randn(P, 4 * C, generator=g) / math.sqrt(4 * C), prec)
    b2 = torch.randn(P, generator=g) * 0.1
    ws = _q(torch.randn(P, C, 1, 1, generator=g) / math.sqrt(C), prec)
    R = [t.clone().requires_grad_() for t in (d, x, w1, b1, w2, b2, ws)]
    hr = F.instance_norm(R[0], eps=1e-5)
    t = F.linear(hr.permute(0, 2, 3, 1), R[2], R[3])
    t = F.linear(F.gelu(t), R[4], R[5]).permute(0, 3, 1, 2)
    y_ref = F.conv2d(R[1], R[6]) + t
    gy = torch.randn(y_ref.shape, generator=g)
    y_ref.backward(gy)
    runs = []
    for folded in (True, False):
        dd, xd = _leaf(d), _leaf(x)
        P_ = [_param(t) for t in (w1, b1, w2, b2, ws)]
        if folded:
            y = HF.pw_mlp(dd, xd, *P_, norm=True)
        else:
            y = HF.pw_mlp(HF.instance_norm(dd), xd, *P_)
        y.backward(gy.to(DEV))
        runs.append([y.detach(), dd.grad, xd.grad] + [p.grad for p in P_])
    tol = TOL[prec]
    names = ("y", "d", "x", "w1", "b1", "w2", "b2", "ws")
    for name, a, r in zip(names, runs[0], [y_ref, R[0].grad, R[1].grad] + [t.grad for t in R[2:]]):
        assert rel(a, r) < (tol if name == "y" else 2 * tol), (name, rel(a, r))
    for name, a, b in zip(names, runs[0], runs[1]):
        assert torch.equal(a, b), (name, rel(a, b))


@pytest.mark.parametrize("N,C,HW", [(2, 64, 256), (3, 128, 4096), (2, 256, 1024), (1, 32, 65536 + 1024)])
@pytest.mark.parametrize("half", HALVES)
def test_instnorm_bf16_output(half, N, C, HW):
    """dsgan_instnorm_fwd_bf16 writes exactly the RNE bf16 rounding of the fp32 InstanceNorm output
    (same statistics, every plane-size kernel variant)."""
    from dsgan_hip import functional as HF_
    HF_.set_precision(half)
    from dsgan_hip import functional as HF
    from dsgan_hip._lib import call, ptr, stream
    g = torch.Generator().manual_seed(C + HW)
    d = (torch.randn(N, C, 1, HW, generator=g) * 3 - 1).to(DEV)
    # the one-workgroup-per-plane fp32 forward (dsgan_instnorm_fwd; instnorm_raw splits few planes)
    y32, m32, r32 = torch.empty_like(d), torch.empty(N * C, device=DEV), torch.empty(N * C, device=DEV)
    call("dsgan_instnorm_fwd", ptr(d), C * HW, None, None, 0, ptr(y32), C * HW, ptr(m32), ptr(r32), N, C, HW, 0, 0.2,
         1e-5, stream())
    yb = torch.empty((N, C, 1, HW), device=DEV, dtype=_hdt(half))
    m, r = torch.empty(N * C, device=DEV), torch.empty(N * C, device=DEV)
    call("dsgan_instnorm_fwd_bf16", ptr(d), C * HW, ptr(yb), C * HW, ptr(m), ptr(r), N, C, HW, 1e-5, stream())
    torch.cuda.synchronize()
    assert torch.equal(yb, y32.to(_hdt(half)))
    assert torch.equal(m, m32) and torch.equal(r, r32)


@pytest.mark.parametrize("w_bf16", [0, 1])
@pytest.mark.parametrize("dy_bf16,dx_bf16,gp", [(0, 1, True), (1, 0, False), (1, 1, True), (0, 0, False)])
@pytest.mark.parametrize("N,M,K,P", [(2, 512, 128, 256), (1, 2048, 256, 128), (2, 96, 64, 384), (1, 1024, 1024, 256)])
@pytest.mark.parametrize("half", HALVES)
def test_pw_dgrad_io(half, w_bf16, dy_bf16, dx_bf16, gp, N, M, K, P):
    """dsgan_pw_dgrad_io: DX = (W^T DY) (* GP) with bf16 DY/DX options vs float64 torch on the
    bf16-rounded operands (the last shape takes the 256-row M tiles)."""
    from dsgan_hip import functional as HF_
    HF_.set_precision(half)
    from dsgan_hip._lib import call, ptr, stream
    g = torch.Generator().manual_seed(M + K + P)
    w = torch.randn(K, M, generator=g) / math.sqrt(K)
    dy = torch.randn(N, K, P, generator=g)
    gpv = torch.rand(N, M, P, generator=g).to(_hdt(half))
    ref = torch.einsum("km,nkp->nmp", _q(w, half).double(), _q(dy, half).double())
    if gp:
        ref = ref * gpv.double()
    dyd = dy.to(DEV).to(_hdt(half)) if dy_bf16 else dy.to(DEV)
    dx = torch.empty((N, M, P), device=DEV, dtype=_hdt(half) if dx_bf16 else torch.float32)
    wd = w.to(DEV).to(_hdt(half)) if w_bf16 else w.to(DEV)
    call("dsgan_pw_dgrad_io", ptr(wd), w_bf16, ptr(dyd), K * P, dy_bf16, ptr(dx), M * P, dx_bf16,
         ptr(gpv.to(DEV)) if gp else None, M * P, M, K, P, N, 0, stream())
    torch.cuda.synchronize()
    got = dx.double().cpu()
    if dx_bf16:
        assert ((got - ref).abs() <= ref.abs() * _ulp(half) + 1e-6).all()
    else:
        assert rel(got, ref) < 1e-5


@pytest.mark.parametrize("dy_bf16,gp", [(0, True), (1, False)])
@pytest.mark.parametrize("half", HALVES)
def test_pw_dgrad_io_wide_tiles(half, dy_bf16, gp):
    """The 256 x 256 x 64 (8-wave) tiles of the bf16 data-grad: a grid of 256 tiles over one image
    (M = 512 rows, 32768 pixels), vs float64 torch on the bf16 operands."""
    from dsgan_hip import functional as HF_
    HF_.set_precision(half)
    from dsgan_hip._lib import call, ptr, stream
    N, M, K, P = 1, 512, 256, 32768
    g = torch.Generator().manual_seed(5)
    w = torch.randn(K, M, generator=g) / math.sqrt(K)
    dy = torch.randn(N, K, P, generator=g)
    gpv = torch.rand(N, M, P, generator=g).to(_hdt(half))
    ref = torch.einsum("km,nkp->nmp", _q(w, half).double(), _q(dy, half).double())
    if gp:
        ref = ref * gpv.double()
    dyd = dy.to(DEV).to(_hdt(half)) if dy_bf16 else dy.to(DEV)
    dx = torch.empty((N, M, P), device=DEV)
    call("dsgan_pw_dgrad_io", ptr(w.to(DEV).to(_hdt(half))), 1, ptr(dyd), K * P, dy_bf16, ptr(dx), M * P, 0,
         ptr(gpv.to(DEV)) if gp else None, M * P, M, K, P, N, 0, stream())
    torch.cuda.synchronize()
    assert rel(dx.double().cpu(), ref) < 1e-5


@pytest.mark.parametrize("a_bf16,b_bf16", [(0, 0), (1, 1), (1, 0), (0, 1)])
@pytest.mark.parametrize("N,M,C,P", [(2, 512, 128, 4096), (16, 64, 512, 1024), (1, 96, 40, 256), (2, 2048, 512, 256)])
@pytest.mark.parametrize("half", HALVES)
def test_pw_wgrad_bias_sums(half, a_bf16, b_bf16, N, M, C, P):
    """dsgan_pw_wgrad_mixed with db: dW += A B^T and db += row sums of A from the staged tiles, split or
    unsplit, fp32 or bf16 A; deterministic (two runs bitwise equal)."""
    from dsgan_hip import functional as HF_
    HF_.set_precision(half)
    from dsgan_hip import functional as HF
    from dsgan_hip._lib import call, ptr, stream
    g = torch.Generator().manual_seed(M + C + P)
    a = torch.randn(N, M, P, generator=g)
    b = torch.randn(N, C, P, generator=g)
    aq, bq = (_q(a, half) if a_bf16 else a), (_q(b, half) if b_bf16 else b)
    ref_w = torch.einsum("nmp,ncp->mc", _q(a, half).double(), _q(b, half).double())
    ref_b = aq.double().sum(dim=(0, 2))
    outs = []
    for _ in range(2):
        w0, b0 = torch.ones(M, C, device=DEV), torch.full((M,), 2.0, device=DEV)
        ad = a.to(DEV).to(_hdt(half)) if a_bf16 else a.to(DEV)
        bd = b.to(DEV).to(_hdt(half)) if b_bf16 else b.to(DEV)
        call("dsgan_pw_wgrad_mixed", ptr(ad), M * P, a_bf16, ptr(bd), C * P, b_bf16, ptr(w0), ptr(b0), M, C, P, N,
             *HF.wsa(HF._pw_ws(M, C, P, N, ad)), stream())
        torch.cuda.synchronize()
        outs.append((w0.cpu(), b0.cpu()))
    assert rel(outs[0][0] - 1.0, ref_w) < 1e-5
    assert rel(outs[0][1] - 2.0, ref_b) < 1e-5
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("N,Cin,H,W,Cout,K,s,p,act", [
    (2, 64, 18, 18, 128, 3, 1, 1, "relu"),       # VGG block (ragged 18x18 vs 8x16 tiles)
    (1, 128, 32, 40, 64, 3, 1, 1, None),
    (2, 32, 34, 30, 64, 4, 2, 1, "lrelu"),       # PatchGAN s2
    (2, 128, 9, 11, 256, 4, 1, 1, None),         # PatchGAN s1 (output 8x10)
    (1, 256, 16, 16, 3 * 32, 3, 1, 1, "relu"),   # M not a multiple of the 128 tile
])
@pytest.mark.parametrize("half", HALVES)
def test_pconv_bf16(half, N, Cin, H, W, Cout, K, s, p, act):
    """Patch-staged conv (pconv.hip): forward and stride-1 data-grad vs the bf16-rounded fp32 conv."""
    from dsgan_hip import functional as HF
    HF.set_precision(half)
    g = torch.Generator().manual_seed(Cin + Cout + K)
    x = _q(torch.randn(N, Cin, H, W, generator=g), half)
    w = _q(torch.randn(Cout, Cin, K, K, generator=g) / math.sqrt(Cin * K * K), half)
    b = torch.randn(Cout, generator=g) * 0.1
    y_ref = F.conv2d(x, w, b, stride=s, padding=p)
    if act == "relu":
        y_ref = F.relu(y_ref)
    elif act == "lrelu":
        y_ref = F.leaky_relu(y_ref, 0.2)
    y = HF.conv_fwd_raw(x.to(DEV), w.to(DEV), b.to(DEV), s, p, act=act)
    assert y.shape == y_ref.shape
    assert rel(y, y_ref) < TOL[half]
    if s == 1:
        gy = _q(torch.randn(y_ref.shape, generator=g), half)
        dx_ref = torch.nn.grad.conv2d_input(x.shape, w, gy, stride=1, padding=p)
        dx = HF.conv_dgrad_raw(gy.to(DEV), w.to(DEV), tuple(x.shape), 1, p)
        assert rel(dx, dx_ref) < TOL[half]
        # fused act' epilogue: dx * relu'(x)
        dxg = HF.conv_dgrad_raw(gy.to(DEV), w.to(DEV), tuple(x.shape), 1, p, gpre=x.to(DEV), gact="relu")
        assert rel(dxg, dx_ref * (x > 0)) < TOL[half]


@pytest.mark.parametrize("N,C,H,W,M,K,s,p", [
    (2, 64, 32, 32, 128, 3, 2, 1),      # ConvT u4 / local.up4 weight-grad class (as the s2 conv)
    (1, 128, 20, 36, 256, 3, 2, 1),     # ragged: 10x18 output pixels vs 4x16 blocks
    (3, 32, 16, 16, 96, 3, 2, 1),       # M not a multiple of the 64 tile
    (2, 32, 34, 36, 64, 4, 2, 1),       # PatchGAN 4x4 s2 (17x18 output)
    (2, 128, 9, 12, 256, 4, 1, 1),      # PatchGAN 4x4 s1 (output 8x11)
    (2, 64, 12, 16, 64, 3, 1, 1),       # 3x3 s1
])
@pytest.mark.parametrize("half", HALVES)
def test_wconv_bf16(half, N, C, H, W, M, K, s, p):
    """Patch-staged weight-grad (wconv.hip) vs torch's conv2d_weight on the bf16-rounded operands;
    accumulates into the existing gradient; deterministic (fixed-order split reduction)."""
    from dsgan_hip import functional as HF
    HF.set_precision(half)
    g = torch.Generator().manual_seed(C + M + K + H)
    x = _q(torch.randn(N, C, H, W, generator=g), half)
    Ho, Wo = (H + 2 * p - K) // s + 1, (W + 2 * p - K) // s + 1
    dy = _q(torch.randn(N, M, Ho, Wo, generator=g), half)
    dw_ref = torch.nn.grad.conv2d_weight(x.double(), (M, C, K, K), dy.double(), stride=s, padding=p)
    w0 = torch.randn(M, C, K, K, generator=g)
    dw = w0.to(DEV)
    HF.IGEMM_TIMER.rec, HF.IGEMM_TIMER.on = [], True
    try:
        HF.conv_wgrad_raw(dy.to(DEV), x.to(DEV), dw, s, p)
    finally:
        HF.IGEMM_TIMER.on = False
    assert HF.IGEMM_TIMER.rec[-1][4] == "wconv_kernel"
    assert rel(dw - w0.to(DEV), dw_ref) < 1e-5
    # channel-slice inputs (batch stride != C*H*W) and determinism
    xb = torch.cat([x, torch.randn(N, 32, H, W, generator=g)], 1).to(DEV)[:, :C]
    dw2 = w0.to(DEV)
    HF.conv_wgrad_raw(dy.to(DEV), xb, dw2, s, p)
    assert torch.equal(dw, dw2)
    # the bias-grad fold (dsgan_wconv_db): the same dw bits, db += sum of the staged fp32 dy tiles
    db0 = torch.randn(M, generator=g)
    dw3, db = w0.to(DEV), db0.to(DEV)
    old = HF.WCONV_DB_FOLD
    HF.WCONV_DB_FOLD = True
    try:
        did_db = HF.conv_wgrad_raw(dy.to(DEV), x.to(DEV), dw3, s, p, db=db)
    finally:
        HF.WCONV_DB_FOLD = old
    assert did_db and torch.equal(dw3, dw)
    assert rel(db - db0.to(DEV), dy.double().sum(dim=(0, 2, 3))) < 1e-6


@pytest.mark.parametrize("N,C,H,W,M,s", [
    (16, 64, 128, 128, 128, 2),    # PatchGAN layer 1 at B = 16 (64 x 64 output)
    (16, 128, 64, 64, 256, 2),     # layer 2 (32 x 32)
    (16, 256, 32, 32, 512, 1),     # layer 3, stride 1 (31 x 31: ragged in both block dimensions)
    (1, 256, 6, 8, 512, 1),        # one partial 16 x 4 pixel block per image: fewer blocks than the split target
    (3, 64, 10, 40, 96, 2),        # 5 x 20 outputs, M not a multiple of the 64-row tile
])
def test_wconv_db_fold_vs_channel_sum(N, C, H, W, M, s):
    """the PatchGAN 4x4 weight-grad's folded bias grad (dsgan_wconv_db) against the
    separate channel-sum kernel, at the step's shapes and at ragged / under-filled ones, with the
    caching allocator's free blocks poisoned with NaN first -- a read of scratch no workgroup
    wrote, or of a D element outside the tensor, turns db non-finite here instead of in training."""
    from dsgan_hip import functional as HF
    HF.set_precision("bf16")
    g = torch.Generator().manual_seed(N + C + H + M)
    Ho, Wo = (H + 2 - 4) // s + 1, (W + 2 - 4) // s + 1
    x = torch.randn(N, C, H, W, generator=g).to(DEV)
    dy = torch.randn(N, M, Ho, Wo, generator=g).to(DEV)
    ws_need = HF._lib.load().dsgan_wconv_workspace(N, C, M, Ho, Wo, 4, 4)
    poison = torch.full((ws_need * 2 + (1 << 20),), float("nan"), device=DEV)
    del poison   # its block returns to the allocator: the next scratch allocation starts as NaN
    dw1, db1 = torch.zeros(M, C, 4, 4, device=DEV), torch.zeros(M, device=DEV)
    old = HF.WCONV_DB_FOLD
    HF.WCONV_DB_FOLD = True
    try:
        assert HF.conv_wgrad_raw(dy, x, dw1, s, 1, db=db1)
    finally:
        HF.WCONV_DB_FOLD = old
    db2, dw2 = torch.zeros(M, device=DEV), torch.zeros(M, C, 4, 4, device=DEV)
    HF.conv_wgrad_raw(dy, x, dw2, s, 1)
    HF.channel_sum_raw(dy, db2)
    torch.cuda.synchronize()
    assert torch.isfinite(db1).all() and torch.isfinite(dw1).all()
    assert torch.equal(dw1, dw2)
    ref = dy.double().sum(dim=(0, 2, 3))
    assert rel(db1, ref) < 1e-6 and rel(db2, ref) < 1e-6, (rel(db1, ref), rel(db2, ref))


@pytest.mark.parametrize("N,C,H,P", [(2, 64, 16, 128), (2, 128, 16, 64), (3, 128, 16, 256), (2, 256, 16, 128),
                                     (1, 128, 32, 64)])
@pytest.mark.parametrize("half", HALVES)
def test_pw_mlp_fused(half, N, C, H, P):
    """bf16 fused MLP kernels (mlp.hip) at every (C, P) they take: forward without the hidden z,
    backward recomputing z and feeding bf16 gelu(z)/dz to the weight-grads."""
    from dsgan_hip import functional as HF, _lib
    HF.set_precision(half)
    assert _lib.load().dsgan_mlp_supported(C, P, H * H) > 0
    g = torch.Generator().manual_seed(7 * C + P)
    h = _q(torch.randn(N, C, H, H, generator=g), half)
    x = _q(torch.randn(N, C, H, H, generator=g), half)
    w1 = _q(torch.randn(4 * C, C, generator=g) / math.sqrt(C), half)
    b1 = torch.randn(4 * C, generator=g) * 0.1
    w2 = _q(torch.randn(P, 4 * C, generator=g) / math.sqrt(4 * C), half)
    b2 = torch.randn(P, generator=g) * 0.1
    ws = _q(torch.randn(P, C, 1, 1, generator=g) / math.sqrt(C), half)
    R = [t.clone().requires_grad_() for t in (h, x, w1, b1, w2, b2, ws)]
    t = F.linear(R[0].permute(0, 2, 3, 1), R[2], R[3])
    t = F.linear(F.gelu(t), R[4], R[5]).permute(0, 3, 1, 2)
    y_ref = F.conv2d(R[1], R[6]) + t
    gy = torch.randn(y_ref.shape, generator=g)
    y_ref.backward(gy)
    hd, xd = _leaf(h), _leaf(x)
    P_ = [_param(t) for t in (w1, b1, w2, b2, ws)]
    y = HF.pw_mlp(hd, xd, *P_)
    y.backward(gy.to(DEV))
    tol = TOL[half]
    assert rel(y, y_ref) < tol
    assert rel(hd.grad, R[0].grad) < 2 * tol
    assert rel(xd.grad, R[1].grad) < 2 * tol
    for name, pd, pr in zip(("w1", "b1", "w2", "b2", "ws"), P_, R[2:]):
        assert rel(pd.grad, pr.grad) < 2 * tol, name


@pytest.mark.parametrize("K", [3, 5, 7, 9])
@pytest.mark.parametrize("N,C,H,W", [(2, 4, 16, 16), (2, 3, 40, 37), (1, 2, 4, 4), (2, 8, 70, 65),
                                     (2, 4, 64, 64), (1, 3, 70, 128), (2, 2, 32, 32), (3, 2, 100, 256)])
def test_dwconv(K, N, C, H, W):
    from dsgan_hip import functional as HF
    g = torch.Generator().manual_seed(K * 100 + C + H)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, 1, K, K, generator=g) / K
    b = torch.randn(C, generator=g)
    xr, wr, br = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    y_ref = F.conv2d(xr, wr, br, padding=K // 2, groups=C)
    gy = torch.randn(y_ref.shape, generator=g)
    y_ref.backward(gy)
    xd, wd, bd = _leaf(x), _param(w), _param(b)
    y = HF.dwconv(xd, wd, bd)
    y.backward(gy.to(DEV))
    assert rel(y, y_ref) < 1e-5
    assert rel(xd.grad, xr.grad) < 1e-5
    assert rel(wd.grad, wr.grad) < 1e-5
    assert rel(bd.grad, br.grad) < 1e-5


@pytest.mark.parametrize("C,H,W", [(128, 128, 128), (512, 64, 64), (1024, 32, 32)])
def test_dwconv_wgrad_prefetch_path(C, H, W):
    """The depthwise weight-grad's next-image prefetch form (dw_wgrad_body PF) runs only where a
    workgroup walks >= 8 images (B = 16 step shapes; the op tests above use N <= 3).  Its dw / db at
    B = 16 against the sum of 16 single-image launches (the plain form, pinned to torch above), per
    tile configuration (W % 128 == 0, W = 64, W = 32)."""
    from dsgan_hip import functional as HF
    N, K = 16, 7
    g = torch.Generator(device=DEV).manual_seed(C + H)
    x = torch.randn(N, C, H, W, device=DEV, generator=g)
    dy = torch.randn(N, C, H, W, device=DEV, generator=g)
    dw, db = torch.zeros(C, 1, K, K, device=DEV), torch.zeros(C, device=DEV)
    HF._dw_wgrad(dy, x, dw, db, K)
    rw, rb = torch.zeros(C, 1, K, K, device=DEV, dtype=torch.float64), torch.zeros(C, device=DEV, dtype=torch.float64)
    for n in range(N):
        w1, b1 = torch.zeros(C, 1, K, K, device=DEV), torch.zeros(C, device=DEV)
        HF._dw_wgrad(dy[n:n + 1].contiguous(), x[n:n + 1].contiguous(), w1, b1, K)
        rw += w1.double()
        rb += b1.double()
    assert rel(dw, rw) < 1e-5 and rel(db, rb) < 1e-5


@pytest.mark.parametrize("N", [16, 2])
def test_multi_dwconv_wgrad_prefetch_path(N):
    """MidMLKA's four-quarter weight-grad at C = 128 @ 128^2: N = 16 takes the prefetch form (16 images
    per workgroup), N = 2 the plain one; the B = 16 grads equal the sum of two B = 8 launches' within
    fp32 summation error, and the N = 2 ones match torch (the four quarter convs)."""
    from dsgan_hip import functional as HF
    C, H = 128, 128
    q = C // 4
    g = torch.Generator(device=DEV).manual_seed(N)
    x = torch.randn(N, C, H, H, device=DEV, generator=g)
    dy = torch.randn(N, C, H, H, device=DEV, generator=g)
    ks = (3, 5, 7, 9)

    def grads(xs, dys):
        ws = torch.empty(max(1, HF._lib.load().dsgan_dwconv_multi_wgrad_workspace(xs.shape[0], q, H, H)), device=DEV)
        gw = [torch.zeros(q, 1, k, k, device=DEV) for k in ks]
        gb = [torch.zeros(q, device=DEV) for _ in ks]
        args = []
        for a_, b_ in zip(gw, gb):
            args += [HF.ptr(a_), HF.ptr(b_)]
        HF.call("dsgan_dwconv_multi_wgrad", HF.ptr(dys), C * H * H, HF.ptr(xs), C * H * H, *args, xs.shape[0], q, H, H,
                HF.ptr(ws), ws.numel(), HF.stream())
        return gw + gb

    got = grads(x, dy)
    if N == 16:
        a, b = grads(x[:8].contiguous(), dy[:8].contiguous()), grads(x[8:].contiguous(), dy[8:].contiguous())
        for t, u, v in zip(got, a, b):
            assert rel(t, u.double() + v.double()) < 1e-5
    else:
        for i, k in enumerate(ks):
            xr = x[:, i * q:(i + 1) * q].detach().cpu().double()
            dr = dy[:, i * q:(i + 1) * q].detach().cpu().double()
            w = torch.zeros(q, 1, k, k, dtype=torch.float64, requires_grad=True)
            b = torch.zeros(q, dtype=torch.float64, requires_grad=True)
            F.conv2d(xr, w, b, padding=k // 2, groups=q).backward(dr)
            assert rel(got[i], w.grad) < 1e-5 and rel(got[4 + i], b.grad) < 1e-5


@pytest.mark.parametrize("K", [3, 7, 9])
@pytest.mark.parametrize("H,W", [(64, 64), (40, 128), (32, 32)])
def test_dwconv_accumulate(K, H, W):
    """Data-grad accumulated into an existing buffer (the Block input's second consumer)."""
    from dsgan_hip import functional as HF
    g = torch.Generator().manual_seed(K + H)
    dy = torch.randn(2, 6, H, W, generator=g)
    w = torch.randn(6, 1, K, K, generator=g) / K
    base = torch.randn(2, 6, H, W, generator=g)
    ref = base + F.conv_transpose2d(dy, w, padding=K // 2, groups=6)
    out = base.to(DEV)
    HF.dwconv_raw(dy.to(DEV), w.to(DEV), None, flip=True, out=out, accumulate=True)
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("act", [None, "gelu", "lrelu"])
@pytest.mark.parametrize("res", [False, True])
# sizes cover every kernel variant: scalar (HW % 4 != 0), float4 wave-per-plane (<= 1K, ragged
# tail), 256-thread cached (<= 4K, <= 16K), 1024-thread cached 64K planes, streaming (> 64K)
# ... and the split forms for < 128 planes of >= 16K pixels (the last three shapes; their 128-plane
# twins take the one-workgroup kernels)
@pytest.mark.parametrize("N,C,H,W", [(2, 3, 4, 4), (2, 5, 33, 31), (1, 2, 80, 80), (2, 4, 16, 16), (2, 3, 36, 20),
                                     (1, 128, 128, 128), (1, 128, 256, 256), (1, 128, 256, 260),
                                     (1, 2, 128, 128), (1, 2, 256, 256), (1, 1, 256, 260)])
def test_instance_norm(act, res, N, C, H, W):
    from dsgan_hip import functional as HF
    g = torch.Generator().manual_seed(C * H + W)
    x = torch.randn(N, C, H, W, generator=g) * 3 + 1
    r = torch.randn(N, C, H, W, generator=g)
    xr = x.clone().requires_grad_()
    rr = r.clone().requires_grad_()
    y_ref = F.instance_norm(xr, eps=1e-5) + (rr if res else 0)
    y_ref = {None: lambda t: t, "gelu": F.gelu, "lrelu": lambda t: F.leaky_relu(t, 0.2)}[act](y_ref)
    gy = torch.randn(y_ref.shape, generator=g)
    y_ref.backward(gy)
    xd, rd = _leaf(x), _leaf(r)
    y = HF.instance_norm(xd, act=act, res=rd if res else None)
    y.backward(gy.to(DEV))
    assert rel(y, y_ref) < 1e-5
    assert rel(xd.grad, xr.grad) < 1e-4
    if res:
        got, ref = rd.grad.cpu(), rr.grad
        if act == "lrelu":
            # LeakyReLU's slope switches at xhat + r = 0: elements within rounding of the kink may take
            # the other slope in either implementation (the 8.5M-element shapes hit a few)
            z = F.instance_norm(x.double(), eps=1e-5) + r.double()
            keep = z.abs() > 1e-5
            got, ref = got[keep], ref[keep]
        assert rel(got, ref) < 1e-5


@pytest.mark.parametrize("k,W", [(2, 48), (2, 50), (4, 48), (8, 48), (16, 48)])
def test_maxpool_indices_bit_exact(k, W):
    """W=48 at k=2 takes the two-outputs-per-thread 16-byte kernel, W=50 the 8-byte one."""
    from dsgan_hip import functional as HF
    g = torch.Generator().manual_seed(k)
    x = torch.randn(2, 3, 32, W, generator=g)
    x[0, 0, :4, :4] = 1.5  # ties: first max in row-major window order wins
    x[1, 2, 5, 7] = float("nan")  # NaN wins its window, as in torch's max_pool2d
    xr = x.clone().requires_grad_()
    y_ref, i_ref = F.max_pool2d(xr, k, return_indices=True)
    gy = torch.randn(y_ref.shape, generator=g)
    y_ref.backward(gy)
    xd = _leaf(x)
    y, idx = HF.max_pool2d(xd, k, return_indices=True)
    y.backward(gy.to(DEV))
    assert torch.allclose(y.cpu(), y_ref.detach(), rtol=0, atol=0, equal_nan=True)  # bit-exact, NaN == NaN
    assert torch.equal(idx.cpu().long(), i_ref)
    assert torch.equal(xd.grad.cpu(), xr.grad)
    # accumulate form (shared gradient buffers): dx += scatter(dy, idx), through the C-ABI
    from dsgan_hip._lib import call, ptr, stream
    N, C, H, _ = x.shape
    base = torch.randn(x.shape, generator=g)
    dxa = base.to(DEV)
    gyd = gy.to(DEV).contiguous()
    call("dsgan_maxpool_bwd", ptr(gyd), C * (H // k) * (W // k), ptr(idx), ptr(dxa), C * H * W, N, C, H, W, k, 1,
         stream())
    assert torch.equal(dxa.cpu(), base + xr.grad)


@pytest.mark.parametrize("levels,H,W", [(4, 32, 64), (4, 16, 128), (3, 48, 64), (2, 16, 64), (1, 16, 64)])
def test_maxpool_pyramid_bit_exact(levels, H, W):
    """The one-pass skip pyramid (dsgan_maxpool_pyr_*): MaxPool2d(2), (4), (8), (16) of one tensor
    against torch's max_pool2d per k -- values and int32 indices bit-exact, with ties spanning the
    sub-windows the k = 8 / 16 levels merge (a tie whose first row-major occurrence is in the
    second sub-window), NaNs (the last NaN of a window wins), an all -inf window and many exact
    ties from a coarse value grid; the backward (every level's grad added in one pass, plain and
    accumulating) against torch's autograd through the separate pools."""
    from dsgan_hip import functional as HF
    from dsgan_hip._lib import call, ptr, stream
    g = torch.Generator().manual_seed(levels * 100 + H + W)
    x = torch.randint(-3, 4, (2, 3, H, W), generator=g).float() * 0.5   # coarse grid: ties everywhere
    x[0, 1] = torch.randn(H, W, generator=g)
    x[0, 0, 0, 3] = 9.0; x[0, 0, 1, 0] = 9.0       # same max in two 2x2 sub-windows: row-major picks (0, 3)
    x[0, 0, 0, 12] = 9.0; x[0, 0, 5, 1] = 9.0      # across the 8x8 sub-windows of a 16x16 window
    x[1, 2, 5, 7] = float("nan"); x[1, 2, 2, 1] = float("nan")   # two NaNs in one window: the later wins
    x[1, 2, 3, 9] = float("nan")
    x[1, 0, :16, :16] = float("-inf")              # all -inf: index = the window's first element
    ks = [2 << lv for lv in range(levels)]
    xr = x.clone().requires_grad_()
    refs = [F.max_pool2d(xr, k, return_indices=True) for k in ks]
    gys = [torch.randn(r[0].shape, generator=g) for r in refs]
    sum((r[0] * gy).sum() for r, gy in zip(refs, gys)).backward()
    xd = _leaf(x)
    ys = HF.max_pool_pyramid(xd, levels)
    outs = HF.MaxPoolPyrFn.apply(x.to(DEV), levels)
    for lv, (y_ref, i_ref) in enumerate(refs):
        assert torch.allclose(ys[lv].detach().cpu(), y_ref.detach(), rtol=0, atol=0, equal_nan=True), ks[lv]
        assert torch.equal(outs[levels + lv].cpu().long(), i_ref), ks[lv]
    sum((y * gy.to(DEV)).sum() for y, gy in zip(ys, gys)).backward()
    assert torch.allclose(xd.grad.cpu().double(), xr.grad.double(), rtol=1e-6, atol=1e-6)
    # accumulate form through the C ABI, with the k = 4 grad absent
    N, C = x.shape[:2]
    base = torch.randn(x.shape, generator=g)
    dxa = base.to(DEV)
    args = []
    for lv in range(4):
        if lv < levels and lv != 1:
            gy = gys[lv].to(DEV).contiguous()
            args += [gy, gy.shape[1] * gy.shape[2] * gy.shape[3], outs[levels + lv]]
        else:
            args += [None, 0, None]
    call("dsgan_maxpool_pyr_bwd", *[ptr(a) if torch.is_tensor(a) or a is None else a for a in args], ptr(dxa),
         C * H * W, levels, N, C, H, W, 1, stream())
    xr2 = x.clone().requires_grad_()
    sum((F.max_pool2d(xr2, ks[lv]) * gys[lv]).sum() for lv in range(levels) if lv != 1).backward()
    assert torch.allclose(dxa.cpu().double(), (base + xr2.grad).double(), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("C,H", [(32, 16), (128, 8), (256, 4)])
def test_mid_tail(C, H):
    """GELU(IN(v * CA(v)) + x) (MixConvNeXtML.py:112-116, CA :18-22) fwd + all grads."""
    from dsgan_hip import functional as HF
    from oracle.dsgan_cpu import ca_fwd
    g = torch.Generator().manual_seed(C)
    N, R = 2, C // 8
    v = torch.randn(N, C, H, H, generator=g)
    x = torch.randn(N, C, H, H, generator=g)
    w1 = torch.randn(R, C, 1, 1, generator=g) / math.sqrt(C)
    w2 = torch.randn(C, R, 1, 1, generator=g) / math.sqrt(R)
    pa = torch.tensor([0.25])
    gy = torch.randn(N, C, H, H, generator=g)

    def ref(dtype):
        T = [t.clone().to(dtype).requires_grad_() for t in (v, x, w1, pa, w2)]
        p = {"a.fc1.weight": T[2], "a.relu1.weight": T[3], "a.fc2.weight": T[4]}
        yr = F.gelu(F.instance_norm(T[0] * ca_fwd(p, "a.", T[0]), eps=1e-5) + T[1])
        yr.backward(gy.to(dtype))
        return yr, T

    y_ref, T = ref(torch.float64)
    y32, T32 = ref(torch.float32)
    vd, xd = _leaf(v), _leaf(x)
    P_ = [_param(t) for t in (w1, pa, w2)]
    y = HF.mid_tail(vd, xd, *P_)
    y.backward(gy.to(DEV))
    assert rel(y, y_ref) < 1e-5
    assert rel(vd.grad, T[0].grad) < 1e-4
    assert rel(xd.grad, T[1].grad) < 1e-5
    # CA weight grads are sums of cancelling terms: bar = 2x torch-fp32's own error vs fp64
    for pd, pr, p32 in zip(P_, T[2:], T32[2:]):
        assert rel(pd.grad, pr.grad) <= max(2 * rel(p32.grad, pr.grad), 1e-5)


@pytest.mark.parametrize("N,C,H,W", [(2, 16, 12, 12),      # per-quarter generic kernels
                                     (2, 32, 32, 32),      # one launch per pass, cfg 3 (W = 32)
                                     (2, 64, 64, 64),      # cfg 2 (W = 64)
                                     (1, 32, 20, 128)])    # cfg 1 (W % 128 == 0), ragged rows
def test_multi_dwconv(N, C, H, W):
    """MidMLKA's four depthwise quarters (X3/X5/X7/X9) fwd + data-grad + weight/bias grads vs torch."""
    from dsgan_hip import functional as HF
    g = torch.Generator().manual_seed(5 + C + W)
    x = torch.randn(N, C, H, W, generator=g)
    q = C // 4
    ws = []
    for k in (3, 5, 7, 9):
        ws += [torch.randn(q, 1, k, k, generator=g) / k, torch.randn(q, generator=g)]
    T = [t.clone().requires_grad_() for t in [x] + ws]
    parts = torch.chunk(T[0], 4, 1)
    y_ref = torch.cat([F.conv2d(parts[i], T[1 + 2 * i], T[2 + 2 * i], padding=k // 2, groups=q)
                       for i, k in enumerate((3, 5, 7, 9))], 1)
    gy = torch.randn(y_ref.shape, generator=g)
    y_ref.backward(gy)
    xd = _leaf(x)
    P_ = [_param(t) for t in ws]
    y = HF.multi_dwconv(xd, *P_)
    y.backward(gy.to(DEV))
    assert rel(y, y_ref) < 1e-5
    assert rel(xd.grad, T[0].grad) < 1e-5
    for pd, pr in zip(P_, T[1:]):
        assert rel(pd.grad, pr.grad) < 1e-5


def test_losses():
    from dsgan_hip import functional as HF
    from oracle import dsgan_cpu as O
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 1, 30, 30, generator=g) * 3
    for t in (0.0, 1.0):
        xr = x.clone().requires_grad_()
        l_ref = O.bce_logits(xr, t)
        l_ref.backward()
        xd = _leaf(x)
        l = HF.bce_with_logits(xd, t)
        l.backward()
        assert abs(l.item() - l_ref.item()) < 1e-5 * abs(l_ref.item())
        assert rel(xd.grad, xr.grad) < 1e-5
    a = torch.randn(2, 3, 40, 40, generator=g)
    b = torch.randn(2, 3, 40, 40, generator=g)
    ar = a.clone().requires_grad_()
    l_ref = torch.mean(torch.abs(ar - b))
    l_ref.backward()
    ad = _leaf(a)
    l = HF.l1_loss(ad, b.to(DEV))
    l.backward()
    assert abs(l.item() - l_ref.item()) < 1e-5
    assert rel(ad.grad, ar.grad) < 1e-6
    # 16-byte path with an n % 4 tail, a large multi-block case, and the unaligned fallback
    for n, off in ((1003, 0), (1 << 22, 0), (1003, 1)):
        u = torch.randn(n + off, generator=g)
        v = torch.randn(n + off, generator=g)
        want = torch.mean(torch.abs(u[off:].double() - v[off:].double())).item()
        got = HF.l1_loss(u.to(DEV)[off:], v.to(DEV)[off:]).item()
        assert abs(got - want) < 1e-5 * want, (n, off, got, want)
    ar = a.clone().requires_grad_()
    l_ref = O.tv_loss(ar)
    l_ref.backward()
    ad = _leaf(a)
    l = HF.tv_loss(ad)
    l.backward()
    assert abs(l.item() - l_ref.item()) < 1e-5 * l_ref.item()
    assert rel(ad.grad, ar.grad) < 1e-6


@pytest.mark.parametrize("shape", [(2, 3, 64, 64), (1, 3, 75, 41), (2, 3, 11, 11)])
def test_ssim_fwd_bwd(shape):
    from dsgan_hip import functional as HF
    from oracle import dsgan_cpu as O
    g = torch.Generator().manual_seed(sum(shape))
    real = torch.rand(shape, generator=g) * 2 - 1
    fake = (real + 0.3 * torch.randn(shape, generator=g)).clamp(-1.2, 1.2)
    fr = fake.clone().requires_grad_()
    s_ref = O.ssim((real.double() + 1) / 2, (fr.double() + 1) / 2)
    s_ref.backward()
    fd = _leaf(fake)
    s = HF.ssim_affine(real.to(DEV), fd, 0.5, 0.5, 1.0)
    s.backward()
    assert abs(s.item() - s_ref.item()) < 2e-5
    assert rel(fd.grad, fr.grad) < 1e-3


def test_ssim_bwd_on_round5_nan_patches():
    """The SSIM backward at the output pixels where round 5's kernel wrote NaN coefficients (configs[4],
    fp16, step 4 of the quality leg: 121 NaN elements of the SSIM input-grad, so the G step was skipped
    and the run drifted from the reference by an MS-SSIM delta of 1.5e-3).  The coefficient maps were
    S * (1 / A1), S * (1 / A2): at an exact zero of A2 = 2 sigma12 + C2, 0 * inf = NaN, although the
    derivative -- the reference's autograd of A / B, DSGAN/MS_SSIM.py:76-88 -- is finite there.  The
    patches (tests/golden/ssim_nan_patch.npz, gen_ssim_nan_patch.py) hold those pixels' 11 x 11 input
    windows; the current kernel must give a finite input-grad that matches float64 autograd."""
    import os
    import numpy as np
    from dsgan_hip import functional as HF
    from oracle import dsgan_cpu as O
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "ssim_nan_patch.npz"))
    real, fake = torch.from_numpy(z["real"]), torch.from_numpy(z["fake"])
    assert real.shape[0] >= 1 and real.shape[1:] == (1, 16, 16)
    for i in range(real.shape[0]):
        r, f = real[i:i + 1], fake[i:i + 1]
        fr = f.double().requires_grad_()
        s_ref = O.ssim((r.double() + 1) / 2, (fr + 1) / 2)
        s_ref.backward()
        fd = _leaf(f)
        s = HF.ssim_affine(r.to(DEV), fd, 0.5, 0.5, 1.0)
        s.backward()
        assert torch.isfinite(fd.grad).all(), i
        assert abs(s.item() - s_ref.item()) < 2e-5
        assert rel(fd.grad, fr.grad) < 1e-3, (i, rel(fd.grad, fr.grad))


def test_ssim_bwd_finite_where_covariance_crosses_minus_c2():
    """Accuracy of the SSIM backward where A2 = 2 sigma12 + C2 and A1 = 2 mu1 mu2 + C1 pass through zero
    (see test_ssim_bwd_on_round5_nan_patches): anti-correlated fields whose local variance sweeps through
    C2 / 2 along W, and a negative fake mean around -C1 / (2 mu1)."""
    from dsgan_hip import functional as HF
    from oracle import dsgan_cpu as O
    g = torch.Generator().manual_seed(77)
    N, C, H, W = 4, 3, 256, 256
    amp = torch.linspace(0.005, 0.05, W).view(1, 1, 1, W)
    noise = F.avg_pool2d(torch.randn(N, C, H + 2, W + 2, generator=g), 3, 1) * 3
    X = 0.75 + amp * noise
    Y = 0.75 - amp * noise + 0.002 * torch.randn(N, C, H, W, generator=g)
    Y[:, 2] = Y[:, 2] - 0.75 - 0.02 * torch.linspace(-1, 1, H).view(H, 1)   # mu2 around -C1 / (2 mu1)
    real, fake = X * 2 - 1, Y * 2 - 1
    fr = fake.clone().double().requires_grad_()
    s_ref = O.ssim((real.double() + 1) / 2, (fr + 1) / 2)
    s_ref.backward()
    fd = _leaf(fake)
    s = HF.ssim_affine(real.to(DEV), fd, 0.5, 0.5, 1.0)
    s.backward()
    bad = int((~torch.isfinite(fd.grad)).sum())
    assert bad == 0, "%d non-finite SSIM input-grad elements" % bad
    assert abs(s.item() - s_ref.item()) < 2e-5
    assert rel(fd.grad, fr.grad) < 1e-3


def test_adam_matches_torch():
    from dsgan_hip.flat import FlatParams, FlatAdam
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Linear(5, 3))
    ref = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Linear(5, 3))
    ref.load_state_dict(net.state_dict())
    flat = FlatParams(net, torch.device(DEV))
    opt = FlatAdam(flat, lr=2e-4, betas=(0.5, 0.999))
    ropt = torch.optim.Adam(ref.parameters(), lr=2e-4, betas=(0.5, 0.999))
    for it in range(5):
        grads = [torch.randn(p.shape) * (10 ** (it - 2)) for p in ref.parameters()]
        for p, gr in zip(ref.parameters(), grads):
            p.grad = gr.clone()
        ropt.step()
        opt.zero_grad()
        for p, gr in zip(net.parameters(), grads):
            p.grad.copy_(gr)
        opt.step()
    for p, q in zip(net.parameters(), ref.parameters()):
        assert torch.allclose(p.detach().cpu(), q.detach(), rtol=1e-6, atol=1e-7)


def test_loss_sum_matches_torch_chain():
    """HF.loss_sum (dsgan_loss_combine) is bit-identical to the torch scalar-op chains it replaces
    in backward_G / backward_D (pix2pix_model.py), values and the grads of every term."""
    from dsgan_hip import functional as HF
    torch.manual_seed(5)
    vals = [torch.rand((), device=DEV) * s for s in (3.0, 0.7, 12.0, 0.01, 1.0)]
    w = (1.0, 100.0, 10.0, 0.37, 1.0)   # gan, (L1), vgg, tv, ss
    for fused in (True, False):
        xs = [v.clone().requires_grad_(True) for v in vals]
        gan, l1, vgg, tv, ss = xs
        if fused:
            loss = HF.loss_sum([(gan, w[0]), (l1, 1.0), (vgg, w[2]), (tv, w[3]), (ss, w[4], 1.0, -1.0)])
        else:
            loss = gan * w[0] + l1 + vgg * w[2] + tv * w[3] + w[4] * (1 - ss)
        (loss * 3.0).backward()
        got = [loss.detach()] + [x.grad for x in xs]
        if fused:
            fused_res = got
        else:
            for a, b in zip(fused_res, got):
                assert torch.equal(a, b), (a, b)
    # the D form: (fake + real) * 0.5
    f, r = (v.clone().requires_grad_(True) for v in vals[:2])
    d = HF.loss_sum([(f, 1.0), (r, 1.0)], 0.5)
    d.backward()
    f2, r2 = (v.clone().requires_grad_(True) for v in vals[:2])
    d2 = (f2 + r2) * 0.5
    d2.backward()
    assert torch.equal(d.detach(), d2.detach()) and torch.equal(f.grad, f2.grad) and torch.equal(r.grad, r2.grad)
    # a disabled term (python 0) is dropped: 0 * w + l1 + ... == l1 + ...
    x = vals[1].clone()
    assert torch.equal(HF.loss_sum([(0, 5.0), (x, 1.0), (vals[2], 2.0)]), 0 * 5.0 + x + vals[2] * 2.0)


@pytest.mark.parametrize("off", [0, 1])          # 0: float4 body + tail, 1: unaligned one-element body
@pytest.mark.parametrize("amp", [False, True])
def test_adam_kernel_paths(off, amp):
    """dsgan_adam / dsgan_adam_amp on a flat buffer of n % 4 == 3 elements, against torch's
    single-tensor Adam formula (fp32, same operation order); the AMP form unscales by state[3] and
    skips the whole update when state[1] != 0."""
    from dsgan_hip._lib import call, ptr, stream
    torch.manual_seed(3)
    n, lr, b1, b2, eps = 300_003, 2e-4, 0.5, 0.999, 1e-8
    base = [torch.randn(n + 1, device=DEV) for _ in range(4)]
    p, g, m, v = (t[off:off + n] for t in base)
    v.abs_()
    scale, step = 1024.0, 3
    p0, m0, v0 = p.clone(), m.clone(), v.clone()
    gr = g / scale if amp else g
    m_ref = m0.lerp(gr, 1 - b1)
    v_ref = v0 * b2 + (1 - b2) * gr * gr
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    p_ref = p0 - (lr / bc1) * (m_ref / (v_ref.sqrt() / (bc2 ** 0.5) + eps))
    if amp:
        st = torch.tensor([scale, 0.0, 0.0, 1.0 / scale, float(step)], device=DEV)
        call("dsgan_adam_amp", ptr(p), ptr(g), ptr(m), ptr(v), n, lr, b1, b2, eps, ptr(st), stream())
    else:
        call("dsgan_adam", ptr(p), ptr(g), ptr(m), ptr(v), n, lr, b1, b2, eps, step, stream())
    torch.cuda.synchronize()
    # (tolerances: one-ulp differences where the kernel contracts a multiply-add into an FMA)
    assert torch.allclose(m, m_ref, rtol=1e-6, atol=1e-7) and torch.allclose(v, v_ref, rtol=1e-6, atol=1e-9)
    assert torch.allclose(p, p_ref, rtol=3e-7, atol=1e-7)   # ~2 ulp of p
    if amp:   # an overflowed step leaves everything untouched
        st = torch.tensor([scale, 1.0, 0.0, 1.0 / scale, float(step)], device=DEV)
        p1, m1, v1 = p.clone(), m.clone(), v.clone()
        call("dsgan_adam_amp", ptr(p), ptr(g), ptr(m), ptr(v), n, lr, b1, b2, eps, ptr(st), stream())
        torch.cuda.synchronize()
        assert torch.equal(p, p1) and torch.equal(m, m1) and torch.equal(v, v1)


@pytest.mark.parametrize("N,Cin,H,Cout", [(2, 64, 16, 256), (2, 36, 16, 200), (3, 132, 32, 68),
                                          (2, 512, 8 * 4, 64), (1, 16, 128, 16)])
@pytest.mark.parametrize("half", HALVES)
def test_pw_gemm_fast_path(half, N, Cin, H, Cout):
    """bf16 1x1 GEMM fast path (pwgemm.hip): fwd(+bias, xact=gelu, accumulate), dgrad(+gelu'
    epilogue), wgrad(+xact) incl. partial M tiles and K % 32 != 0, vs fp32 torch on bf16-rounded
    operands."""
    from dsgan_hip import functional as HF
    from dsgan_hip import _lib
    HF.set_precision(half)
    g = torch.Generator().manual_seed(Cin * 7 + Cout)
    x = torch.randn(N, Cin, H, H, generator=g)
    w = torch.randn(Cout, Cin, 1, 1, generator=g) / math.sqrt(Cin)
    b = torch.randn(Cout, generator=g) * 0.1
    y0 = torch.randn(N, Cout, H, H, generator=g)
    xq, wq = _q(F.gelu(x), half), _q(w, half)
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    assert _lib.load().dsgan_pw_supported(0, Cout, Cin, H * H, 0, Cin * H * H, wd.data_ptr(), xd.data_ptr())
    # fwd with activation-on-load and accumulate
    y = y0.clone().to(DEV)
    HF.conv_fwd_raw(xd, wd, bd, 1, 0, out=y, accumulate=True, xact="gelu")
    ref = F.conv2d(xq, wq, b) + y0
    assert rel(y, ref) < 1e-2
    # dgrad with gelu' epilogue
    dy = torch.randn(N, Cout, H, H, generator=g)
    z = torch.randn(N, Cin, H, H, generator=g)
    dx = HF.conv_dgrad_raw(dy.to(DEV), wd, tuple(x.shape), 1, 0, gpre=z.to(DEV), gact="gelu")
    zr = z.clone().requires_grad_()
    gz = torch.autograd.grad(F.gelu(zr), zr, torch.ones_like(z))[0]
    ref = F.conv_transpose2d(_q(dy, half), wq) * gz
    assert rel(dx, ref) < 1e-2
    # wgrad with activation-on-load
    dw = torch.zeros_like(wd)
    HF.conv_wgrad_raw(dy.to(DEV), xd, dw, 1, 0, xact="gelu")
    ref = torch.einsum("bmhw,bkhw->mk", _q(dy, half), xq).view_as(w)
    assert rel(dw, ref) < 1e-2
    HF.set_precision("fp32")


@pytest.mark.parametrize("N,Cin,H,W,Cout,K,s,p", [
    (2, 64, 18, 18, 128, 3, 1, 1),     # VGG-like
    (2, 32, 20, 13, 200, 3, 1, 1),     # ragged pixels, partial M tile
    (2, 32, 32, 32, 64, 4, 2, 1),      # PatchGAN s2
    (2, 128, 9, 9, 256, 4, 1, 1),      # PatchGAN s1 (31x31-like odd outputs)
    (2, 64, 16, 16, 3, 3, 1, 1),       # G head (M = 3)
])
@pytest.mark.parametrize("half", HALVES)
def test_tap_conv_bf16(half, N, Cin, H, W, Cout, K, s, p):
    """Tap-major bf16 conv (tconv.hip): fwd, stride-1 dgrad (flipped kernel) and stride-2 dgrad
    (parity classes) vs fp32 torch on bf16-rounded operands."""
    from dsgan_hip import functional as HF
    HF.set_precision(half)
    g = torch.Generator().manual_seed(Cin + Cout + K + H)
    x = _q(torch.randn(N, Cin, H, W, generator=g), half)
    w = _q(torch.randn(Cout, Cin, K, K, generator=g) / math.sqrt(Cin * K * K), half)
    b = torch.randn(Cout, generator=g) * 0.1
    y = HF.conv_fwd_raw(x.to(DEV), w.to(DEV), b.to(DEV), s, p, act="relu")
    assert rel(y, F.relu(F.conv2d(x, w, b, stride=s, padding=p))) < 1e-2
    Ho, Wo = y.shape[2], y.shape[3]
    dy = _q(torch.randn(N, Cout, Ho, Wo, generator=g), half)
    gp = torch.randn(N, Cin, H, W, generator=g)
    if Cout % 32 == 0:
        dx = HF.conv_dgrad_raw(dy.to(DEV), w.to(DEV), (N, Cin, H, W), s, p, gpre=gp.to(DEV), gact="lrelu")
        xr = torch.zeros(N, Cin, H, W, requires_grad=True)
        ref = torch.autograd.grad(F.conv2d(xr, w, None, stride=s, padding=p), xr, dy)[0]
        ref = ref * torch.where(gp > 0, 1.0, 0.2)
        assert rel(dx, ref) < 1e-2
    HF.set_precision("fp32")


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
def test_perceptual_l1_fused(prec):
    """VGG16 perceptual term as one node (PerceptualL1Fn): loss and d(loss)/d(fake) vs torch's
    conv2d/relu/max_pool2d/l1_loss chain (DSGAN/models/vgg.py:30-42, pix2pix_model.py:182-186)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ds-gan_amd"))
    from dsgan_hip import functional as HF
    from models.vgg import Vgg16
    HF.set_precision(prec)
    torch.manual_seed(3)
    vgg = Vgg16(seed=11).to(DEV)
    g = torch.Generator().manual_seed(5)
    fake = _q(torch.randn(2, 3, 32, 48, generator=g), prec)
    real = _q(torch.randn(2, 3, 32, 48, generator=g), prec)
    blocks = [(pool, [(w.detach().cpu(), b.detach().cpu()) for w, b in convs]) for pool, convs in vgg.loss_blocks()]

    def ref_feats(x):
        feats, h = [], x
        for pool, convs in blocks:
            if pool:
                h = F.max_pool2d(h, 2)
            for w, b in convs:
                h = F.relu(F.conv2d(h, _q(w, prec), b, padding=1))
            feats.append(h)
        return feats
    fr = fake.clone().requires_grad_()
    f, r = ref_feats(fr), [t.detach() for t in ref_feats(real)]
    loss_ref = F.l1_loss(f[1], r[1]) + F.l1_loss(f[2], r[2]) + F.l1_loss(f[3], r[3]) + F.l1_loss(f[0], r[0])
    loss_ref.backward()
    fd = _leaf(fake)
    rfe = vgg.loss_features(real.to(DEV))
    loss = vgg.perceptual_l1(fd, rfe)
    loss.backward()
    if prec == "fp32":
        assert abs(loss.item() - loss_ref.item()) <= 1e-5 * abs(loss_ref.item())
        assert rel(fd.grad, fr.grad) < 2e-5
    else:
        # bf16 activations move sign(f - r) and the ReLU masks against an fp32 chain, so the
        # bf16 node is checked against the unfused HIP chain on the same kernels/rounding
        # (Conv2dFn + MaxPoolFn + L1Fn autograd), and its loss against fp32 at the bf16 bar.
        assert abs(loss.item() - loss_ref.item()) <= 2e-2 * abs(loss_ref.item())
        fu = _leaf(fake)
        f = vgg(fu)
        rr = list(rfe)
        lu = HF.l1_loss(f[1], rr[1]) + HF.l1_loss(f[2], rr[2]) + HF.l1_loss(f[3], rr[3]) + HF.l1_loss(f[0], rr[0])
        lu.backward()
        assert abs(loss.item() - lu.item()) <= 1e-5 * abs(lu.item())
        assert rel(fd.grad, fu.grad) < 1e-3


@pytest.mark.parametrize("N,Cout,Cin,Hi,Wi,K,H,W", [
    (2, 64, 32, 8, 9, 3, 16, 18),        # ConvT 3x3/s2/op1 (ragged 8x9 grid vs 8x16 tiles)
    (1, 128, 96, 16, 16, 3, 32, 32),     # M not a multiple of the 64 tile
    (2, 64, 32, 17, 18, 4, 34, 36),      # data-grad of the PatchGAN 4x4/s2 conv
    (2, 128, 64, 16, 16, 4, 32, 32),
])
@pytest.mark.parametrize("half", HALVES)
def test_pconvt_bf16(half, N, Cout, Cin, Hi, Wi, K, H, W):
    """pconvt.hip: the stride-2 data-grad / ConvTranspose with all four output parities in one
    launch, vs torch's conv2d_input on bf16-rounded operands; bias, act'(gpre) and accumulate."""
    from dsgan_hip import functional as HF
    HF.set_precision(half)
    g = torch.Generator().manual_seed(Cout + Cin + K + Hi)
    dy = _q(torch.randn(N, Cout, Hi, Wi, generator=g), half)
    w = _q(torch.randn(Cout, Cin, K, K, generator=g) / math.sqrt(Cout * K * K / 4), half)
    b = torch.randn(Cin, generator=g) * 0.1
    dx_ref = torch.nn.grad.conv2d_input((N, Cin, H, W), w.double(), dy.double(), stride=2, padding=1)
    HF.IGEMM_TIMER.rec, HF.IGEMM_TIMER.on = [], True
    try:
        dx = HF.conv_dgrad_raw(dy.to(DEV), w.to(DEV), (N, Cin, H, W), 2, 1, bias=b.to(DEV))
    finally:
        HF.IGEMM_TIMER.on = False
    assert HF.IGEMM_TIMER.rec[-1][4] == "pconvt_kernel"
    assert rel(dx, dx_ref + b.double().view(1, -1, 1, 1)) < 1e-5
    pre = torch.randn(N, Cin, H, W, generator=g)
    y0 = torch.randn(N, Cin, H, W, generator=g)
    out = y0.to(DEV)
    HF.conv_dgrad_raw(dy.to(DEV), w.to(DEV), (N, Cin, H, W), 2, 1, gpre=pre.to(DEV), gact="lrelu", out=out,
                      accumulate=True)
    want = y0.double() + dx_ref * torch.where(pre > 0, 1.0, 0.2).double()
    assert rel(out, want) < 1e-5


@pytest.mark.parametrize("shape", [(2, 3, 5, 7), (3, 4, 16, 16), (2, 8, 64, 64)])
def test_add_n_and_cat(shape):
    """AddNFn / CatFn (float4 and scalar forms): exact sums and channel concatenation."""
    from dsgan_hip import functional as HF
    g = torch.Generator().manual_seed(shape[1] * shape[2])
    xs = [torch.randn(shape, generator=g) for _ in range(3)]
    y = HF.add_n(*[t.to(DEV) for t in xs])
    assert torch.equal(y.cpu(), (xs[0] + xs[1]) + xs[2])
    b = torch.randn(shape[0], 2, shape[2], shape[3], generator=g)
    ad, bd = _leaf(xs[0]), _leaf(b)
    c = HF.cat_channels(ad, bd)
    assert torch.equal(c.detach().cpu(), torch.cat([xs[0], b], 1))
    gy = torch.randn(c.shape, generator=g)
    c.backward(gy.to(DEV))
    assert torch.equal(ad.grad.cpu(), gy[:, :shape[1]]) and torch.equal(bd.grad.cpu(), gy[:, shape[1]:])


@pytest.mark.parametrize("shape", [(2, 3, 8, 8), (2, 4, 32, 32)])
def test_instance_norm_cat(shape):
    """upSample tail: cat(GELU(IN(x)), skip) with the IN writing into the concatenation."""
    from dsgan_hip import functional as HF
    g = torch.Generator().manual_seed(shape[1])
    x = torch.randn(shape, generator=g) * 2 + 0.5
    sk = torch.randn(shape[0], 5, shape[2], shape[3], generator=g)
    xr, sr = x.clone().requires_grad_(), sk.clone().requires_grad_()
    y_ref = torch.cat([F.gelu(F.instance_norm(xr, eps=1e-5)), sr], 1)
    gy = torch.randn(y_ref.shape, generator=g)
    y_ref.backward(gy)
    xd, sd = _leaf(x), _leaf(sk)
    y = HF.instance_norm_cat(xd, sd, act="gelu")
    y.backward(gy.to(DEV))
    assert rel(y, y_ref) < 1e-5
    assert rel(xd.grad, xr.grad) < 1e-4
    assert torch.equal(sd.grad.cpu(), sr.grad)


@pytest.mark.parametrize("half", HALVES)
@pytest.mark.parametrize("act,res", [("gelu", False), ("gelu", True), (None, True)])
@pytest.mark.parametrize("N,C,H,W", [(2, 64, 16, 16), (1, 32, 64, 64), (2, 96, 32, 36), (1, 4, 256, 256)])
def test_instnorm_bwd_h_is_rounded_fp32_backward(half, act, res, N, C, H, W):
    """dsgan_instnorm_bwd_h: its 16-bit dx is the RNE rounding of dsgan_instnorm_bwd's fp32 dx
    (bit for bit), dres is identical, dxsum the per-plane sum of the fp32 dx."""
    from dsgan_hip import functional as HF
    from dsgan_hip._lib import call, ptr, stream
    HF.set_precision(half)
    g = torch.Generator().manual_seed(C + H)
    x = (torch.randn(N, C, H, W, generator=g) * 2 + 0.3).to(DEV)
    dy = torch.randn(N, C, H, W, generator=g).to(DEV)
    r = torch.randn(N, C, H, W, generator=g).to(DEV) if res else None
    _, mean, rstd = HF.instnorm_raw(x, None, r, act)
    # the one-workgroup-per-plane fp32 backward (dsgan_instnorm_bwd; instnorm_bwd_raw splits few planes)
    HW = H * W
    dx32, dres32 = torch.empty_like(x), (torch.empty_like(x) if res else None)
    call("dsgan_instnorm_bwd", ptr(dy), C * HW, ptr(x), C * HW, None, ptr(r), C * HW, ptr(mean), ptr(rstd), ptr(dx32),
         C * HW, ptr(dres32), C * HW, None, N, C, HW, HF.ACT[act], 0.2, 1e-5, stream())
    dxh = torch.empty((N, C, H, W), device=DEV, dtype=_hdt(half))
    dsum = torch.empty(N * C, device=DEV)
    dres = torch.empty_like(x) if res else None
    call("dsgan_instnorm_bwd_h", ptr(dy), C * HW, ptr(x), C * HW, ptr(r), C * HW, ptr(mean), ptr(rstd), ptr(dxh),
         C * HW, ptr(dsum), ptr(dres), C * HW, N, C, HW, HF.ACT[act], 0.2, 1e-5, stream())
    torch.cuda.synchronize()
    assert torch.equal(dxh.cpu(), dx32.to(_hdt(half)).cpu())
    if res:
        assert torch.equal(dres.cpu(), dres32.cpu())
    ref = dx32.double().sum((2, 3)).flatten()
    scale = dx32.double().abs().sum((2, 3)).flatten()
    assert ((dsum.double() - ref).abs() <= 1e-6 * scale + 1e-30).all()


@pytest.mark.parametrize("half", HALVES)
@pytest.mark.parametrize("cat", [True, False])
@pytest.mark.parametrize("N,Ci,Co,H", [(2, 128, 64, 16), (2, 256, 128, 8), (1, 1024, 512, 16), (2, 64, 32, 24)])
def test_convt_norm_fused_matches_unfused(half, cat, N, Ci, Co, H):
    """ConvTNormFn (16-bit ConvT output grad from the IN backward, tconv / wconv reading it as
    16-bit operands) vs conv_transpose3s2 + instance_norm(_cat) (fp32 grad, rounded on load):
    the same output bits; dx bitwise (same tconv tiles and K order on the same operand values);
    dW to fp32 summation order (the 16-bit-X wconv plans twice the pixel splits); the bias grad
    (the ConvT output grad sums to ~0 under the InstanceNorm) to the fp32 rounding of its sum."""
    from dsgan_hip import functional as HF
    HF.set_precision(half)
    g = torch.Generator().manual_seed(Ci + Co + H + int(cat))
    x = torch.randn(N, Ci, H, H, generator=g)
    w = torch.randn(Ci, Co, 3, 3, generator=g) / math.sqrt(Ci * 9)
    b = torch.randn(Co, generator=g) * 0.1
    o = torch.randn(N, 48 if cat else Co, 2 * H, 2 * H, generator=g)
    gy = torch.randn(N, Co + (48 if cat else 0), 2 * H, 2 * H, generator=g).to(DEV)
    outs = []
    for fused in (True, False):
        xd, od, wd, bd = _leaf(x), _leaf(o), _param(w), _param(b)
        if fused:
            assert HF._convt_norm_fused(xd, wd, od, cat)
            y = HF.ConvTNormFn.apply(xd, wd, bd, od, "gelu", cat)
        else:
            t = HF.conv_transpose3s2(xd, wd, bd)
            y = HF.instance_norm_cat(t, od, "gelu") if cat else HF.instance_norm(t, "gelu", od)
        y.backward(gy)
        torch.cuda.synchronize()
        outs.append((y.detach().cpu(), xd.grad.cpu(), wd.grad.cpu(), bd.grad.cpu(), od.grad.cpu()))
    (y1, dx1, dw1, db1, do1), (y2, dx2, dw2, db2, do2) = outs
    assert torch.equal(y1, y2)
    assert torch.equal(dx1, dx2)
    assert torch.equal(do1, do2)
    assert rel(dw1, dw2) < 1e-5
    # |bias grad| ~ fp32 rounding of a near-cancelling sum: bar on the scale of the summands
    t_scale = gy[:, :Co].abs().double().sum((0, 2, 3)).cpu()
    assert ((db1.double() - db2.double()).abs() <= 1e-5 * t_scale).all()


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("N,C,P,H,Ci", [(2, 64, 64, 32, 128),     # fused MLP kernels (mlp.hip)
                                        (2, 256, 128, 16, 256),   # unfused bf16 g / gp path
                                        (2, 3, 64, 32, 128)])     # tiny block (c1: pw_small2)
def test_cat_slot_in_place(prec, N, C, P, H, Ci):
    """HF.CatSlot (the decoder skip written in place, MixConvNeXtML.py:229-236): the Block tail
    writes R into the slot's tail, the ConvT + IN node fills only the head and returns the whole
    buffer.  Against the same graph with a freshly allocated R and a copied skip: every output and
    gradient bitwise (the kernels see the same values, only R's batch stride differs)."""
    from dsgan_hip import functional as HF
    HF.set_precision(prec)
    g = torch.Generator().manual_seed(C + P + H)
    d = torch.randn(N, C, H, H, generator=g)
    x = torch.randn(N, C, H, H, generator=g)
    w1 = torch.randn(4 * C, C, generator=g) / math.sqrt(C)
    b1 = torch.randn(4 * C, generator=g) * 0.1
    w2 = torch.randn(P, 4 * C, generator=g) / math.sqrt(4 * C)
    b2 = torch.randn(P, generator=g) * 0.1
    ws = torch.randn(P, C, 1, 1, generator=g) / math.sqrt(C)
    u = torch.randn(N, Ci, H // 2, H // 2, generator=g)
    wt = torch.randn(Ci, P, 3, 3, generator=g) / math.sqrt(Ci * 9)
    bt = torch.randn(P, generator=g) * 0.1
    gy = torch.randn(N, 2 * P, H, H, generator=g).to(DEV)
    gp = torch.randn(N, P, H // 2, H // 2, generator=g).to(DEV)
    outs = []
    for use_slot in (False, True):
        dd, xd, ud = _leaf(d), _leaf(x), _leaf(u)
        Q = [_param(t) for t in (w1, b1, w2, b2, ws, wt, bt)]
        slot = HF.CatSlot(N, P, P, H, H, dd) if use_slot else None
        R = HF.share(HF.pw_mlp(dd, xd, *Q[:5], norm=True, slot=slot))
        if use_slot:
            assert slot.holds(R, P) and R.stride(0) == 2 * P * H * H
        pooled = HF.max_pool2d(R, 2)
        y = HF.convt_norm(ud, Q[5], Q[6], R, act="gelu", cat=True, slot=slot)
        if use_slot:
            assert y.data_ptr() == slot.buf.data_ptr()
        # fresh upstream grads per run: R's shared grad buffer adopts its slice of gy and the
        # max-pool backward accumulates into it
        torch.autograd.backward([y, pooled], [gy.clone(), gp.clone()])
        torch.cuda.synchronize()
        outs.append([y.detach().cpu(), pooled.detach().cpu(), dd.grad.cpu(), xd.grad.cpu(), ud.grad.cpu()]
                    + [q.grad.cpu() for q in Q])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("N,C,P,H", [(2, 64, 64, 32), (2, 256, 128, 16), (2, 3, 64, 32)])
def test_pw_mlp_acc_in_place(prec, N, C, P, H):
    """pw_mlp(..., acc=A) (the G tail uc4(U4) + Loc, MixConvNeXtML.py:236-239): the block output
    summed into A in place by the shortcut GEMM's epilogue, A returned dirty.  Against block + A as
    a separate add: the forward to fp32 rounding (one add moved ahead of the MLP's), A's grad is the
    upstream grad, every other grad bitwise (the backward never reads A)."""
    from dsgan_hip import functional as HF
    HF.set_precision(prec)
    g = torch.Generator().manual_seed(C + P + H + 7)
    ins = [torch.randn(N, C, H, H, generator=g) for _ in range(2)]
    prm = [torch.randn(4 * C, C, generator=g) / math.sqrt(C), torch.randn(4 * C, generator=g) * 0.1,
           torch.randn(P, 4 * C, generator=g) / math.sqrt(4 * C), torch.randn(P, generator=g) * 0.1,
           torch.randn(P, C, 1, 1, generator=g) / math.sqrt(C)]
    a0 = torch.randn(N, P, H, H, generator=g)
    gy = torch.randn(N, P, H, H, generator=g).to(DEV)
    outs = []
    for fused in (False, True):
        dd, xd, ad = _leaf(ins[0]), _leaf(ins[1]), _leaf(a0)
        Q = [_param(t) for t in prm]
        a = ad * 1.0   # a non-leaf A, as the local branch's output is
        y = HF.pw_mlp(dd, xd, *Q, norm=True, acc=a) if fused else HF.add_n(HF.pw_mlp(dd, xd, *Q, norm=True), a)
        if fused:
            assert y.data_ptr() == a.data_ptr()
        y.backward(gy.clone())
        torch.cuda.synchronize()
        outs.append([y.detach().cpu(), ad.grad.cpu(), dd.grad.cpu(), xd.grad.cpu()] + [q.grad.cpu() for q in Q])
    (y1, da1, *r1), (y2, da2, *r2) = outs
    assert rel(y2, y1) < 1e-6
    assert torch.equal(da1, gy.cpu()) and torch.equal(da2, gy.cpu())
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)


@pytest.mark.parametrize("w_bf16,x_bf16", [(0, 0), (1, 1), (1, 0)])
@pytest.mark.parametrize("M,K,P,nb", [(2048, 512, 4096, 2), (1024, 256, 1024, 3), (256, 64, 256, 2), (4096, 1024, 1024, 1),
                                      (96, 40, 256, 2)])
@pytest.mark.parametrize("half", HALVES)
def test_pw_fwd_io_bf16_outputs(half, w_bf16, x_bf16, M, K, P, nb):
    """pwconv1 of the unfused MLP blocks (MixConvNeXtML.py:221-223): g = gelu(W x + b) and
    gp = gelu'(W x + b) written bf16 through the LDS-staged epilogue, vs torch on the same bf16
    operands (one bf16 ulp)."""
    from dsgan_hip import functional as HF_
    HF_.set_precision(half)
    import dsgan_hip
    from dsgan_hip._lib import call, ptr, stream
    from dsgan_hip import functional as HF
    dsgan_hip.require_gpu()
    g = torch.Generator().manual_seed(M + K)
    x = torch.randn(nb, K, P, generator=g).cuda()
    w = (torch.randn(M, K, generator=g) / K ** 0.5).cuda()
    b = torch.randn(M, generator=g).cuda()
    y = torch.empty(nb, M, P, device="cuda", dtype=_hdt(half))
    gp = torch.empty_like(y)
    wd, xd = (w.to(_hdt(half)) if w_bf16 else w), (x.to(_hdt(half)) if x_bf16 else x)
    call("dsgan_pw_fwd_io", ptr(wd), w_bf16, ptr(xd), K * P, x_bf16, ptr(y), M * P, 1, ptr(gp), M * P, 1, ptr(b), M, K,
         P, nb, HF.ACT["gelu"], 0, 0.2, stream())
    z = torch.einsum("mk,bkp->bmp", w.to(_hdt(half)).double(), x.to(_hdt(half)).double()) + b.double().view(1, M, 1)
    zz = z.clone().requires_grad_(True)
    torch.nn.functional.gelu(zz).sum().backward()
    ref_g, ref_gp = torch.nn.functional.gelu(z), zz.grad
    torch.cuda.synchronize()
    for got, ref in ((y, ref_g), (gp, ref_gp)):
        got = got.double()
        assert ((got - ref.cuda()).abs() <= ref.cuda().abs() * 2 ** -7 + 1e-3).all()


@pytest.mark.parametrize("N,K,M,H,W", [(2, 64, 3, 8, 256), (1, 20, 2, 4, 512)])
def test_thin3_accumulate_and_strides(N, K, M, H, W):
    """thin3.hip fwd / dgrad accumulate into (and read) channel slices of larger buffers."""
    from dsgan_hip import functional as HF
    HF.set_precision("fp32")
    g = torch.Generator().manual_seed(K * 7 + M)
    xb = torch.randn(N, K + 4, H, W, generator=g)          # x = channels 4.. of a bigger tensor
    x = xb[:, 4:]
    w = torch.randn(M, K, 3, 3, generator=g) / math.sqrt(9 * K)
    b = torch.randn(M, generator=g)
    y0 = torch.randn(N, M + 2, H, W, generator=g)
    y = y0.to(DEV)
    HF.conv_fwd_raw(xb.to(DEV)[:, 4:], w.to(DEV), b.to(DEV), 1, 1, out=y[:, 1:1 + M], accumulate=True)
    ref = y0.clone()
    ref[:, 1:1 + M] += F.conv2d(x, w, b, padding=1)
    assert rel(y, ref) < 1e-5
    dy = torch.randn(N, M, H, W, generator=g)
    dx0 = torch.randn(N, K + 4, H, W, generator=g)
    dx = dx0.to(DEV)
    HF.conv_dgrad_raw(dy.to(DEV), w.to(DEV), (N, K, H, W), 1, 1, out=dx[:, 4:], accumulate=True)
    refx = dx0.clone()
    refx[:, 4:] += torch.nn.grad.conv2d_input((N, K, H, W), w, dy, padding=1)
    assert rel(dx, refx) < 1e-5
    dw = torch.randn(M, K, 3, 3, generator=g)
    dwd = dw.to(DEV)
    HF.conv_wgrad_raw(dy.to(DEV), xb.to(DEV)[:, 4:], dwd, 1, 1)
    refw = dw + torch.nn.grad.conv2d_weight(x, (M, K, 3, 3), dy, padding=1)
    assert rel(dwd, refw) < 1e-5


@pytest.mark.parametrize("half", HALVES)
@pytest.mark.parametrize("N,M,K,P", [(16, 64, 1024, 256), (16, 512, 1024, 256), (4, 256, 512, 256), (2, 96, 640, 128)])
def test_pw_split_k(half, N, M, K, P):
    """Split-K of under-filled pointwise FWD / DGRAD launches (dsgan_pw_fd_workspace > 0): fp32
    partials per K split, then the finishing pass with every epilogue form -- FWD bias + GELU +
    fp32 pre-activation + accumulate, FWD GELU pair into 16-bit g / g', DGRAD gelu'(fp32 pre)
    (+accumulate), DGRAD * 16-bit gp into a 16-bit dz -- vs float64 torch on the 16-bit operands,
    and against the same launches with the split turned off (dsgan_pw_tune(0, 0))."""
    from dsgan_hip import functional as HF
    from dsgan_hip import _lib
    from dsgan_hip._lib import call, ptr, stream
    HF.set_precision(half)
    lib = _lib.load()
    assert lib.dsgan_pw_fd_workspace(0, M, K, P, N) > 0 and lib.dsgan_pw_fd_workspace(1, M, K, P, N) > 0
    hd = _hdt(half)
    g = torch.Generator().manual_seed(M * 3 + K + P)
    x = torch.randn(N, K, P, generator=g)
    w = torch.randn(M, K, generator=g) / math.sqrt(K)
    b = torch.randn(M, generator=g) * 0.1
    y0 = torch.randn(N, M, P, generator=g)
    dy = torch.randn(N, K, P, generator=g)
    z = torch.randn(N, M, P, generator=g)
    gpv = torch.rand(N, M, P, generator=g).to(hd)
    wT = w.t().contiguous()                                   # DGRAD: W[K'=M][M'=K] -> here [K][M]
    # every device operand is held by a name for the whole test: a temporary freed right after ptr()
    # would be handed to the next allocation on the stream before the kernel reads it
    xd, wd, bd, dyd, zd = x.to(DEV), w.to(DEV), b.to(DEV), dy.to(DEV), z.to(DEV)
    xh, wh, wTd, gpd = xd.to(hd), wd.to(hd), wT.to(DEV), gpv.to(DEV)
    wTh = wTd.to(hd)
    wss = {mode: torch.empty(lib.dsgan_pw_fd_workspace(mode, M, K, P, N), device=DEV) for mode in (0, 1)}

    def ws(mode):
        return wss[mode]

    def runs():
        out = {}
        # FWD fp32 operands: y = gelu(W x + b) + y0, pre-activation to ypre
        y, pre = y0.to(DEV), torch.empty(N, M, P, device=DEV)
        call("dsgan_pw_gemm", 0, ptr(wd), 0, ptr(xd), K * P, ptr(y), M * P, ptr(bd), ptr(pre), M * P, None, 0,
             M, N * P, K, P, N, HF.ACT["gelu"], 0, 0, 1, 0.2, *HF.wsa(ws(0)), stream())
        out["fwd"], out["pre"] = y, pre
        # FWD 16-bit in / GELU pair out
        gg, gp = torch.empty(N, M, P, device=DEV, dtype=hd), torch.empty(N, M, P, device=DEV, dtype=hd)
        call("dsgan_pw_fwd_io_ws", ptr(wh), 1, ptr(xh), K * P, 1, ptr(gg), M * P, 1, ptr(gp), M * P, 1,
             ptr(bd), M, K, P, N, HF.ACT["gelu"], 0, 0.2, *HF.wsa(ws(0)), stream())
        out["g"], out["gp"] = gg, gp
        # DGRAD fp32: dx = (W^T dy) * gelu'(z) + y0  (W stored [K][M] as the layer's [out][in] weight)
        dx = y0.to(DEV)
        call("dsgan_pw_gemm", 1, ptr(wTd), 0, ptr(dyd), K * P, ptr(dx), M * P, None, None, 0, ptr(zd), M * P,
             M, N * P, K, P, N, 0, HF.ACT["gelu"], 0, 1, 0.2, *HF.wsa(ws(1)), stream())
        out["dgrad"] = dx
        # DGRAD 16-bit: dz = (W^T dy) * gp, 16-bit out
        dz = torch.empty(N, M, P, device=DEV, dtype=hd)
        call("dsgan_pw_dgrad_io_ws", ptr(wTh), 1, ptr(dyd), K * P, 0, ptr(dz), M * P, 1, ptr(gpd),
             M * P, M, K, P, N, 0, *HF.wsa(ws(1)), stream())
        out["dz"] = dz
        torch.cuda.synchronize()
        return {k: v.double().cpu() for k, v in out.items()}

    split = runs()
    old = lib.dsgan_pw_tune(0, 0)
    try:
        whole = runs()
    finally:
        lib.dsgan_pw_tune(0, old)
    qx, qw, qdy = _q(x, half).double(), _q(w, half).double(), _q(dy, half).double()
    zr = torch.einsum("mk,nkp->nmp", qw, qx) + b.double().view(1, M, 1)
    zz = zr.clone().requires_grad_(True)
    F.gelu(zz).sum().backward()
    ref = {"pre": zr, "fwd": F.gelu(zr) + y0.double(), "g": F.gelu(zr), "gp": zz.grad}
    zg = z.double().clone().requires_grad_(True)
    F.gelu(zg).sum().backward()
    t = torch.einsum("mk,nkp->nmp", qw, qdy)
    ref["dgrad"] = t * zg.grad + y0.double()
    ref["dz"] = t * gpv.double()
    for k in ("pre", "fwd", "dgrad"):
        assert rel(split[k], ref[k]) < 1e-5, k
    for k in ref:   # the unsplit launch sums K in another order: fp32 rounding, or a 16-bit ulp
        assert rel(split[k], whole[k]) < (1e-5 if k in ("pre", "fwd", "dgrad") else 4 * _ulp(half)), k
    for k in ("g", "gp", "dz"):
        assert ((split[k] - ref[k]).abs() <= ref[k].abs() * 2 * _ulp(half) + 1e-3).all(), k
    HF.set_precision("fp32")


@pytest.mark.parametrize("half", HALVES)
def test_weight_copy_refresh_batched(half):
    """bump_weight_generation(params) rebuilds every cached 16-bit copy of those parameters
    (tap-major modes 0-2, plain casts) in one dsgan_wtrans_multi launch: bitwise equal to the
    per-copy launches, and the cache then hits without a rebuild."""
    from dsgan_hip import functional as HF
    from dsgan_hip._lib import call, ptr, stream
    HF.set_precision(half)
    g = torch.Generator().manual_seed(11)
    w4 = torch.nn.Parameter(torch.randn(96, 40, 3, 3, generator=g).to(DEV))
    w4b = torch.nn.Parameter(torch.randn(64, 128, 4, 4, generator=g).to(DEV))
    w2 = torch.nn.Parameter(torch.randn(300, 77, generator=g).to(DEV))
    copies = [HF._wtrans_bf16(w4, m) for m in (0, 1, 2)] + [HF._wtrans_bf16(w4b, 1), HF.bf16_weight(w2)]
    with torch.no_grad():   # an in-place optimizer update (the fused Adam is invisible to torch's versions)
        for p in (w4, w4b, w2):
            p.copy_(torch.randn(p.shape, generator=g).to(DEV))
    HF.bump_weight_generation([w4, w4b, w2])
    again = [HF._wtrans_bf16(w4, m) for m in (0, 1, 2)] + [HF._wtrans_bf16(w4b, 1), HF.bf16_weight(w2)]
    assert all(a.data_ptr() == b.data_ptr() for a, b in zip(copies, again))   # refreshed in place, cache hits
    ref = []
    for w, m in ((w4, 0), (w4, 1), (w4, 2), (w4b, 1)):
        wb = torch.empty(w.numel(), device=DEV, dtype=_hdt(half))
        call("dsgan_conv_wtrans_bf16", ptr(w), ptr(wb), *w.shape, m, stream())
        ref.append(wb)
    ref.append(w2.detach().to(_hdt(half)))
    torch.cuda.synchronize()
    for a, b in zip(again, ref):
        assert torch.equal(a.view(-1).view(torch.int16), b.view(-1).view(torch.int16))
    HF.set_precision("fp32")


@pytest.mark.parametrize("shape", [(2, 3, 80, 80), (2, 5, 7, 9), (2, 4, 64, 64), (3, 6, 16, 16)])
def test_plane_stats_fwd_bwd(shape):
    """Channel-attention plane statistics (CA avg/max pool, MixConvNeXtML.py:5-22): mean, max and the
    FIRST argmax (torch's tie rule; a NaN wins and sticks) of every (n, c) plane, 16-byte and scalar
    forms; the backward dx += davg/HW + (i == argmax) dmx."""
    from dsgan_hip._lib import call, ptr, stream
    N, C, H, W = shape
    HW = H * W
    g = torch.Generator().manual_seed(HW + C)
    x = torch.randn(N, C, H, W, generator=g)
    x[0, 0].view(-1)[[5, HW - 3]] = 7.0                  # tie: the first index wins
    x[1, C - 1].view(-1)[[HW // 2, HW // 2 + 1]] = float("nan")
    xd = x.to(DEV)
    avg = torch.empty(N * C, device=DEV)
    mx = torch.empty(N * C, device=DEV)
    am = torch.empty(N * C, device=DEV, dtype=torch.int32)
    call("dsgan_plane_stats", ptr(xd), C * HW, ptr(avg), ptr(mx), ptr(am), N, C, HW, stream())
    davg = torch.randn(N * C, generator=g)
    dmx = torch.randn(N * C, generator=g)
    dx0 = torch.randn(N, C, H, W, generator=g)
    dx = dx0.to(DEV)
    dd, dm = davg.to(DEV), dmx.to(DEV)
    call("dsgan_plane_stats_bwd", ptr(dd), ptr(dm), ptr(am), ptr(dx), C * HW, N, C, HW, stream())
    torch.cuda.synchronize()
    flat = x.view(N * C, HW)
    ref_mx, ref_am = flat.max(dim=1)
    nan_rows = torch.isnan(flat).any(dim=1)
    assert torch.equal(am.cpu()[~nan_rows].long(), ref_am[~nan_rows])
    assert torch.equal(mx.cpu()[~nan_rows], ref_mx[~nan_rows])
    for r in torch.nonzero(nan_rows).view(-1).tolist():   # first NaN index, value NaN
        assert torch.isnan(mx.cpu()[r]) and am.cpu()[r].item() == int(torch.nonzero(torch.isnan(flat[r]))[0])
    ok = ~nan_rows
    assert torch.allclose(avg.cpu()[ok], flat[ok].double().mean(dim=1).float(), rtol=1e-5, atol=1e-6)
    ref_dx = dx0.view(N * C, HW) + (davg / HW).view(-1, 1)
    ref_dx[torch.arange(N * C), am.cpu().long()] += dmx
    assert torch.allclose(dx.cpu().view(N * C, HW), ref_dx, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("n", [1027, 4 * 300000 + 2])   # a scalar tail (n % 4 != 0); many check blocks
def test_loss_scaler_state_machine(n):
    """dsgan_amp_check / amp_update (adam.hip:135-169) against GradScaler's rule
    (torch/amp/grad_scaler.py _amp_update_scale_): overflow -> skip, scale x backoff, clean count
    reset; `interval` clean steps -> scale x growth; applied-step count only on clean steps.  The
    non-finite element sits in the scalar tail, in the vector body and is a nan; the skipped
    optimizer step leaves params / moments untouched.  Also the unit-scale guard (bf16 mode)."""
    from dsgan_hip.amp import LossScaler
    from dsgan_hip.flat import FlatAdam
    sc = LossScaler(DEV, init_scale=2.0 ** 10, growth_factor=2.0, backoff_factor=0.5, growth_interval=3)
    g = torch.randn(n, device=DEV) * 1e-3
    scale, clean, applied = 2.0 ** 10, 0, 0
    bad_at = {1: n - 1, 4: n // 3, 5: 0}           # step -> poisoned index (tail, body, first)
    for step in range(10):
        gg = g.clone()
        if step in bad_at:
            gg[bad_at[step]] = float("nan") if step == 4 else float("inf")
        sc.check(gg)
        torch.cuda.synchronize()
        st = sc.state.cpu().tolist()
        skip = step in bad_at
        assert st[1] == (1.0 if skip else 0.0), (step, st)
        assert st[3] == 1.0 / scale, (step, st)
        if skip:
            scale, clean = scale * 0.5, 0
        else:
            applied += 1
            clean += 1
            if clean >= 3:
                scale, clean = scale * 2.0, 0
        assert st[0] == scale and st[2] == clean and st[4] == applied, (step, st, scale, clean, applied)

    # the optimizer on a skipped step: nothing moves
    class _Flat:
        pass
    fl = _Flat()
    fl.data = torch.randn(4099, device=DEV)
    fl.grad = torch.randn(4099, device=DEV)
    fl.grad[4098] = float("inf")
    fl.numel = 4099
    fl.params = [torch.nn.Parameter(fl.data)]
    gs = LossScaler.guard(DEV)
    opt = FlatAdam(fl, scaler=gs)
    p0 = fl.data.clone()
    gs.check(fl.grad)
    opt.step()
    torch.cuda.synchronize()
    assert torch.equal(fl.data, p0) and not opt.m.any() and not opt.v.any()
    assert gs.skipped_last() and gs.get_scale() == 1.0 and gs.skipped_steps(1) == 1
    # a clean step under the guard = plain Adam (scale exactly 1, step count 1)
    fl.grad[4098] = 0.5
    gs.check(fl.grad)
    opt.step()
    torch.cuda.synchronize()
    ref = p0.clone()
    call_adam = torch.optim.Adam([torch.nn.Parameter(ref)], lr=2e-4, betas=(0.9, 0.999), eps=1e-8)
    call_adam.param_groups[0]["params"][0].grad = fl.grad.clone()
    call_adam.step()
    assert gs.get_scale() == 1.0 and gs.applied_steps() == 1
    assert rel(fl.data, call_adam.param_groups[0]["params"][0].detach()) < 1e-6


@pytest.mark.parametrize("half", HALVES)
@pytest.mark.parametrize("N,H", [(2, 16), (3, 32)])
def test_mlp_bwd_c256_forms_bitwise(half, N, H):
    """The three forms of the C = 256 MLP backward with g / dz out (mlp.hip: register-staged weights,
    LDS-DMA weight ring, the ring with precomputed addresses; dsgan_mlp_tune key 0) give the same bits for dh, g, dz and the per-32-pixel
    dz sums -- and dh matches the fp32 chain within the 16-bit bar."""
    import dsgan_hip
    from dsgan_hip import _lib
    from dsgan_hip._lib import call, ptr, stream
    lib = _lib.load()
    dsgan_hip.set_precision(half)
    C, P, HW = 256, 128, H * H
    C4 = 4 * C
    hd = _hdt(half)
    g0 = torch.Generator(device=DEV).manual_seed(11)
    h = torch.randn(N, C, HW, device=DEV, generator=g0).to(hd)
    dy = torch.randn(N, P, HW, device=DEV, generator=g0)
    w1 = (torch.randn(C4, C, device=DEV, generator=g0) / C ** 0.5).to(hd)
    w2 = (torch.randn(P, C4, device=DEV, generator=g0) / C4 ** 0.5).to(hd)
    b1 = torch.randn(C4, device=DEV, generator=g0) * 0.1
    old = lib.dsgan_mlp_tune(0, -1)
    outs = {}
    try:
        for mode in (1, 0, 2):
            lib.dsgan_mlp_tune(0, mode)
            dh = torch.full((N, C, HW), float("nan"), device=DEV)
            gg = torch.empty(N, C4, HW, device=DEV, dtype=hd)
            dz = torch.empty_like(gg)
            bs = torch.full((N * HW // 32, C4), float("nan"), device=DEV)
            call("dsgan_mlp_bwd", ptr(h), C * HW, 1, ptr(dy), P * HW, ptr(w1), ptr(b1), ptr(w2), ptr(dh), C * HW,
                 ptr(gg), ptr(dz), ptr(bs), N, C, P, HW, stream())
            torch.cuda.synchronize()
            outs[mode] = (dh, gg, dz, bs)
    finally:
        lib.dsgan_mlp_tune(0, old)
    for mode in (0, 2):
        for a, b in zip(outs[mode], outs[1]):
            assert torch.equal(a, b), mode
    # value check of dh against the fp32 chain on the same 16-bit operands
    hf, w1f, w2f = h.float(), w1.float(), w2.float()
    z = torch.einsum("kc,nch->nkh", w1f, hf) + b1[None, :, None]
    t = torch.einsum("pk,nph->nkh", w2f, dy)
    gp = 0.5 * (1 + torch.erf(z / math.sqrt(2))) + z * torch.exp(-0.5 * z * z) / math.sqrt(2 * math.pi)
    dzr = (t * gp).to(hd).float()
    dhr = torch.einsum("kc,nkh->nch", w1f, dzr)
    assert rel(outs[1][0], dhr) < 3 * _ulp(half)


@pytest.mark.parametrize("half", HALVES)
@pytest.mark.parametrize("form", ["fwd16", "fwd32", "fwd_gelu_pair", "dgrad32", "dgrad16", "wgrad"])
@pytest.mark.parametrize("ring", [3, 2])
def test_pw_wide_dma_ring_bitwise(half, form, ring):
    """The LDS-DMA ring form of the wide 16-bit-operand pointwise GEMMs (pw_impl.h NS = 4, planner
    knob dsgan_pw_tune(9)) against the register-staged wide kernel: the same MFMAs in the same order,
    so FWD / DGRAD outputs and WGRAD weight grads are bitwise equal; the WGRAD bias sums (row sums of
    the staged A tiles) within 1e-6.  Full 256 x 256 tiles, >= 256 of them."""
    import dsgan_hip
    from dsgan_hip import _lib, functional as HF
    from dsgan_hip._lib import call, ptr, stream
    lib = _lib.load()
    dsgan_hip.set_precision(half)
    hd = _hdt(half)
    g0 = torch.Generator(device=DEV).manual_seed(5)
    NB, HW = 4, 128 * 128
    M, K = (512, 256) if form != "wgrad" else (256, 512)
    w = (torch.randn(M, K, device=DEV, generator=g0) / K ** 0.5).to(hd)
    bias = torch.randn(M, device=DEV, generator=g0)
    x = torch.randn(NB, K, HW, device=DEV, generator=g0).to(hd)
    dy = torch.randn(NB, M, HW, device=DEV, generator=g0).to(hd)
    old = lib.dsgan_pw_tune(9, -1)

    def run(dma):
        lib.dsgan_pw_tune(9, dma)
        if form.startswith("fwd"):
            y16 = form != "fwd32"
            y = torch.empty(NB, M, HW, device=DEV, dtype=hd if y16 else torch.float32)
            gp = torch.empty(NB, M, HW, device=DEV, dtype=hd) if form == "fwd_gelu_pair" else None
            ws = torch.empty(max(1, lib.dsgan_pw_fd_workspace(0, M, K, HW, NB)), device=DEV)
            call("dsgan_pw_fwd_io_ws", ptr(w), 1, ptr(x), K * HW, 1, ptr(y), M * HW, int(y16), ptr(gp),
                 M * HW if gp is not None else 0, 1 if gp is not None else 0, ptr(bias), M, K, HW, NB,
                 1 if gp is not None else 0, 0, 0.2, *HF.wsa(ws), stream())
            return [y] + ([gp] if gp is not None else [])
        if form.startswith("dgrad"):   # dx[K] = W^T dy[M]: W [M][K] is the [in][out] operand
            y16 = form == "dgrad16"
            dx = torch.empty(NB, K, HW, device=DEV, dtype=hd if y16 else torch.float32)
            ws = torch.empty(max(1, lib.dsgan_pw_fd_workspace(1, K, M, HW, NB)), device=DEV)
            call("dsgan_pw_dgrad_io_ws", ptr(w), 1, ptr(dy), M * HW, 1, ptr(dx), K * HW, int(y16), None, 0, K, M,
                 HW, NB, 0, *HF.wsa(ws), stream())
            return [dx]
        dw = torch.zeros(M, K, device=DEV)
        db = torch.zeros(M, device=DEV)
        ws = torch.empty(max(1, lib.dsgan_pw_wgrad_workspace(M, K, HW, NB)), device=DEV)
        call("dsgan_pw_wgrad_mixed", ptr(dy), M * HW, 1, ptr(x), K * HW, 1, ptr(dw), ptr(db), M, K, HW, NB,
             *HF.wsa(ws), stream())
        return [dw, db]
    try:
        ref = run(0)
        got = run(ring)
        torch.cuda.synchronize()
    finally:
        lib.dsgan_pw_tune(9, old)
    if form == "wgrad":
        assert torch.equal(got[0], ref[0])
        assert rel(got[1], ref[1]) < 1e-6
    else:
        for a, b in zip(got, ref):
            assert torch.equal(a, b)
    # and the values: fp32 chain on the same 16-bit operands
    if form == "fwd32":
        r = torch.einsum("mk,nkp->nmp", w.float(), x.float()) + bias[None, :, None]
        assert rel(got[0], r) < 1e-5
