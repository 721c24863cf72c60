"""The channel-blocked bf16 VGG16 pass (csrc/vggconv.hip) vs torch fp32 references of the same
ops (DSGAN/models/vgg.py:15-42; loss DSGAN/models/pix2pix_model.py:180-186).

Operands are rounded to bf16 before the torch reference runs, so a conv differs from it only by
fp32 summation order (bar 1e-5 relative on fp32 outputs; one bf16 ulp on bf16 outputs).  MaxPool
values and window argmax are bit-exact; the tap backward is exact up to its bf16 output rounding.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _hf():
    import dsgan_hip
    from dsgan_hip import functional as HF
    dsgan_hip.require_gpu()
    return HF


def to_cb16(t):
    N, C, H, W = t.shape
    return t.reshape(N, C // 16, 16, H, W).permute(0, 1, 3, 4, 2).contiguous()


def from_cb16(t):
    N, Cb, H, W, _ = t.shape
    return t.permute(0, 1, 4, 2, 3).reshape(N, Cb * 16, H, W)


def bf(t):
    return t.to(torch.bfloat16).float()


HALVES = ["bf16", "fp16"]


def _hdt(half):
    return torch.float16 if half == "fp16" else torch.bfloat16


def _ulp(half):
    return 2.0 ** -11 if half == "fp16" else 2.0 ** -8


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()


# (N, Cin, Cout, H, W): the VGG layer shapes at 256^2 (batch 2) and a 512-channel layer at 64^2
SHAPES = [(2, 64, 64, 64, 64), (2, 64, 128, 32, 64), (2, 128, 128, 32, 32), (2, 128, 256, 32, 32),
          (2, 256, 256, 16, 32), (1, 256, 512, 32, 32), (2, 512, 512, 8, 32), (3, 64, 64, 12, 96)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("out_f32", [True, False])
@pytest.mark.parametrize("half", HALVES)
def test_vconv_forward(half, shape, out_f32):
    HT = _hdt(half)
    bf = lambda v: v.to(HT).float()  # noqa: E731 -- this half type
    from dsgan_hip import functional as HF_
    HF_.set_precision(half)
    HF = _hf()
    from dsgan_hip._lib import call, ptr, stream
    N, Ci, Co, H, W = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = bf(torch.relu(torch.randn(N, Ci, H, W, generator=g)))
    w = torch.randn(Co, Ci, 3, 3, generator=g) * (2.0 / (9 * Ci)) ** 0.5
    b = torch.randn(Co, generator=g) * 0.1
    ref = torch.relu(F.conv2d(x.double(), bf(w).double(), b.double(), padding=1))
    xd, wd, bd = to_cb16(x).cuda().to(HT), w.cuda(), b.cuda()
    y = torch.empty((N, Co // 16, H, W, 16), device="cuda", dtype=torch.float32 if out_f32 else HT)
    HF._vconv(xd, HF._vgg_wt(wd, 0), bd, None, y, N, Ci, Co, H, W, True, "fwd")
    torch.cuda.synchronize()
    got = from_cb16(y.float().cpu())
    if out_f32:
        assert rel(got, ref) < 1e-5, rel(got, ref)
    else:
        assert ((got.double() - ref).abs() <= ref.abs() * _ulp(half) + 1e-6).all()


@pytest.mark.parametrize("shape", SHAPES[:6])
@pytest.mark.parametrize("masked", [True, False])
@pytest.mark.parametrize("half", HALVES)
def test_vconv_dgrad(half, shape, masked):
    """The data-grad form: dx = conv_transpose(dy, W) [* (a_below > 0)] with the flipped /
    transposed weights of dsgan_vconv_wtrans(dgrad=1)."""
    HT = _hdt(half)
    bf = lambda v: v.to(HT).float()  # noqa: E731 -- this half type
    from dsgan_hip import functional as HF_
    HF_.set_precision(half)
    HF = _hf()
    N, Ci, Co, H, W = shape
    g = torch.Generator().manual_seed(7 + sum(shape))
    dy = bf(torch.randn(N, Co, H, W, generator=g) * 1e-3)
    w = torch.randn(Co, Ci, 3, 3, generator=g) * (2.0 / (9 * Ci)) ** 0.5
    below = bf(torch.relu(torch.randn(N, Ci, H, W, generator=g)))
    ref = F.conv_transpose2d(dy.double(), bf(w).double(), padding=1)
    if masked:
        ref = ref * (below > 0)
    out = torch.empty((N, Ci // 16, H, W, 16), device="cuda", dtype=HT)
    HF._vconv(to_cb16(dy).cuda().to(HT), HF._vgg_wt(w.cuda(), 1), None,
              to_cb16(below).cuda().to(HT) if masked else None, out, N, Co, Ci, H, W, False, "dgrad")
    torch.cuda.synchronize()
    got = from_cb16(out.float().cpu())
    # absolute floor: fp16 outputs below 2^-14 are subnormal (fixed spacing 2^-24)
    floor = 2.0 ** -24 if half == "fp16" else 1e-9
    assert ((got.double() - ref).abs() <= ref.abs() * _ulp(half) + floor).all()


@pytest.mark.parametrize("half", HALVES)
@pytest.mark.parametrize("N,H,W", [(2, 32, 64), (1, 9, 14), (3, 20, 36)])   # HW % 64 == 0 (scalar weights) or not
def test_conv1_forward_and_dgrad(half, N, H, W):
    HT = _hdt(half)
    bf = lambda v: v.to(HT).float()  # noqa: E731 -- this half type
    from dsgan_hip import functional as HF_
    HF_.set_precision(half)
    HF = _hf()
    from dsgan_hip._lib import call, ptr, stream
    g = torch.Generator().manual_seed(3 + H * W)
    x = torch.rand(N, 3, H, W, generator=g) * 2 - 1
    w = torch.randn(64, 3, 3, 3, generator=g) * 0.3
    b = torch.randn(64, generator=g) * 0.1
    ref = torch.relu(F.conv2d(x.double(), w.double(), b.double(), padding=1))
    y = torch.empty((N, 4, H, W, 16), device="cuda", dtype=HT)
    xd, wd, bd = x.cuda(), w.cuda(), b.cuda()   # named: a temporary freed after ptr() could be re-handed out
    call("dsgan_vgg_conv1_fwd", ptr(xd), 3 * H * W, ptr(wd), ptr(bd), ptr(y), N, H, W, stream())
    d = bf(torch.randn(N, 64, H, W, generator=g) * 1e-3)
    dx = torch.empty((N, 3, H, W), device="cuda")
    dd = to_cb16(d).cuda().to(HT)
    call("dsgan_vgg_conv1_dgrad", ptr(dd), ptr(wd), ptr(dx), 3 * H * W, N, H, W, stream())
    torch.cuda.synchronize()
    got = from_cb16(y.float().cpu())
    assert ((got.double() - ref).abs() <= ref.abs() * _ulp(half) + 1e-6).all()
    dref = F.conv_transpose2d(d.double(), w.double(), padding=1)
    assert rel(dx.cpu(), dref) < 1e-6


@pytest.mark.parametrize("half", HALVES)
@pytest.mark.parametrize("shape", [(2, 32, 16, 24), (3, 48, 34, 18), (1, 16, 2, 2)])
def test_maxpool_l1_fused(half, shape):
    """dsgan_cb16_maxpool_l1: the same pooled values and argmax bits as dsgan_cb16_maxpool, and the
    tap's perceptual L1 mean |f - r| (from the pool's read of f) against float64; a ragged last
    workgroup (thread count not a multiple of 256) included."""
    HT = _hdt(half)
    from dsgan_hip import functional as HF_
    HF_.set_precision(half)
    _hf()
    from dsgan_hip._lib import call, ptr, stream, load
    g = torch.Generator().manual_seed(11)
    N, C, H, W = shape
    f = torch.relu(torch.randn(N, C, H, W, generator=g))
    f[:, :, ::3, ::2] = 0.0
    r = torch.relu(torch.randn(N, C, H, W, generator=g))
    fd, rd = to_cb16(f).cuda(), to_cb16(r).cuda()
    y0 = torch.empty((N, C // 16, H // 2, W // 2, 16), device="cuda", dtype=HT)
    i0 = torch.empty(y0.shape, device="cuda", dtype=torch.uint8)
    call("dsgan_cb16_maxpool", ptr(fd), ptr(y0), ptr(i0), N, C, H, W, stream())
    y1, i1 = torch.empty_like(y0), torch.empty_like(i0)
    part = torch.empty(load().dsgan_cb16_maxpool_l1_parts(N, C, H, W), device="cuda")
    out = torch.full((2,), -1.0, device="cuda")
    codes = torch.empty(fd.shape, device="cuda", dtype=torch.uint8)
    call("dsgan_cb16_maxpool_l1", ptr(fd), ptr(rd), ptr(y1), ptr(i1), ptr(codes), ptr(out), ptr(part), part.numel(),
         N, C, H, W, stream())
    torch.cuda.synchronize()
    assert torch.equal(y0.cpu(), y1.cpu()) and torch.equal(i0.cpu(), i1.cpu())
    ref = (f.double() - r.double()).abs().mean().item()
    assert abs(out[0].item() - ref) <= 2e-6 * ref, (out[0].item(), ref)
    assert out[1].item() == -1.0   # one scalar written
    with pytest.raises(RuntimeError):   # undersized partial scratch is refused
        call("dsgan_cb16_maxpool_l1", ptr(fd), ptr(rd), ptr(y1), ptr(i1), None, ptr(out), ptr(part), part.numel() - 1,
             N, C, H, W, stream())
    # the tap backward from the codes = the one from f and r, bit for bit
    dpool = (torch.randn(N, C, H // 2, W // 2, generator=g) * 1e-3)
    dpd = to_cb16(dpool).cuda().to(HT)
    gsc = torch.tensor([0.75], device="cuda")
    d0 = torch.empty(fd.shape, device="cuda", dtype=HT)
    d1 = torch.empty_like(d0)
    call("dsgan_cb16_tap_bwd", ptr(dpd), ptr(i0), ptr(fd), ptr(rd), ptr(d0), N, C, H, W, ptr(gsc), stream())
    call("dsgan_cb16_tap_bwd_codes", ptr(dpd), ptr(i0), ptr(codes), ptr(d1), N, C, H, W, ptr(gsc), stream())
    torch.cuda.synchronize()
    assert torch.equal(d0.view(torch.int16).cpu(), d1.view(torch.int16).cpu())


@pytest.mark.parametrize("half", HALVES)
def test_maxpool_and_tap_bwd(half):
    """MaxPool2d(2) value + window argmax (first max wins, as torch) and the tapped-layer
    backward (maxpool backward + L1 backward) * ReLU' against torch autograd."""
    HT = _hdt(half)
    bf = lambda v: v.to(HT).float()  # noqa: E731 -- this half type
    from dsgan_hip import functional as HF_
    HF_.set_precision(half)
    _hf()
    from dsgan_hip._lib import call, ptr, stream
    g = torch.Generator().manual_seed(5)
    N, C, H, W = 2, 32, 16, 24
    f = torch.relu(torch.randn(N, C, H, W, generator=g))
    f[:, :, ::3, ::2] = 0.0                      # ties among zeros, as post-ReLU features have
    r = torch.relu(torch.randn(N, C, H, W, generator=g))
    fd, rd = to_cb16(f).cuda(), to_cb16(r).cuda()
    y = torch.empty((N, C // 16, H // 2, W // 2, 16), device="cuda", dtype=HT)
    idx = torch.empty(y.shape, device="cuda", dtype=torch.uint8)
    call("dsgan_cb16_maxpool", ptr(fd), ptr(y), ptr(idx), N, C, H, W, stream())
    ref, ridx = F.max_pool2d(f, 2, return_indices=True)
    torch.cuda.synchronize()
    assert torch.equal(from_cb16(y.float().cpu()), bf(ref))
    rh, rw = ridx // W, ridx % W
    win = ((rh % 2) * 2 + (rw % 2)).to(torch.uint8)
    assert torch.equal(from_cb16(idx.cpu()), win)
    # backward: loss = gsc * L1(f, r) + <dpool, maxpool(f)>, grad at the pre-ReLU input
    dpool = bf(torch.randn(N, C, H // 2, W // 2, generator=g) * 1e-3)
    # fp16: the loss-scaled magnitude the fp16 mode feeds this kernel (dsgan_hip.amp: x 2^16), so
    # the gradients stay in the normal fp16 range
    gsc = torch.tensor([0.75 * (2.0 ** 16 if half == "fp16" else 1.0)])
    pre = f.clone().requires_grad_(True)
    out = torch.relu(pre)
    loss = gsc * torch.mean(torch.abs(out - r)) + (F.max_pool2d(out, 2) * dpool).sum()
    loss.backward()
    d = torch.empty(fd.shape, device="cuda", dtype=HT)
    call("dsgan_cb16_tap_bwd", ptr(to_cb16(dpool).cuda().to(HT)), ptr(idx), ptr(fd), ptr(rd), ptr(d), N, C,
         H, W, ptr(gsc.cuda()), stream())
    torch.cuda.synchronize()
    got = from_cb16(d.float().cpu())
    refg = pre.grad * (f > 0)
    assert ((got.double() - refg.double()).abs() <= refg.abs().double() * _ulp(half) + 1e-12).all()


def test_perceptual_cb16_matches_nchw_path():
    """The whole perceptual term at 256x256 in bf16: the CB16 pass vs the NCHW bf16 pass
    (loss value and grad w.r.t. fake_B) and vs an fp32 torch reference of vgg.py."""
    HF = _hf()
    from models.vgg import Vgg16
    vgg = Vgg16().cuda()
    g = torch.Generator().manual_seed(9)
    real = (torch.rand(2, 3, 256, 256, generator=g) * 2 - 1).cuda()
    fake = (real + 0.3 * torch.randn(2, 3, 256, 256, generator=g).cuda()).clamp(-1, 1)
    res = {}
    with HF.precision("bf16"):
        for path in ("cb16", "nchw"):
            blocks = vgg.loss_blocks()
            rf = HF.vgg_features_cb16(real, blocks)[0] if path == "cb16" else HF.vgg_features_raw(real, blocks)[0]
            fk = fake.clone().requires_grad_(True)
            loss = HF.perceptual_l1(fk, blocks, rf)
            loss.backward()
            torch.cuda.synchronize()
            res[path] = (loss.item(), fk.grad.detach().cpu())
    # fp32 torch reference of the reference's forward
    fr = fake.detach().cpu().float().requires_grad_(True)

    def feats(x):
        out, h = [], x
        for bi, (pool, convs) in enumerate(vgg.loss_blocks()):
            if pool:
                h = F.max_pool2d(h, 2)
            for w, b in convs:
                h = torch.relu(F.conv2d(h, w.detach().cpu().float(), b.detach().cpu().float(), padding=1))
            out.append(h)
        return out
    with torch.no_grad():
        rr = feats(real.cpu().float())
    ff = feats(fr)
    lref = sum(torch.mean(torch.abs(a - b)) for a, b in zip((ff[1], ff[2], ff[3], ff[0]), (rr[1], rr[2], rr[3], rr[0])))
    lref.backward()
    l_cb, g_cb = res["cb16"]
    l_nc, g_nc = res["nchw"]
    gref = fr.grad
    cos = lambda a, b: (a.double().flatten() @ b.double().flatten() / (a.double().norm() * b.double().norm())).item()
    print("perceptual: loss cb16 %.6f nchw %.6f fp32 %.6f | grad rel cb16-fp32 %.4f nchw-fp32 %.4f cb16-nchw %.4f"
          " cos %.5f %.5f" % (l_cb, l_nc, lref.item(), rel(g_cb, gref), rel(g_nc, gref), rel(g_cb, g_nc),
                              cos(g_cb, gref), cos(g_nc, gref)))
    assert abs(l_cb - l_nc) <= 1e-4 * abs(l_nc), (l_cb, l_nc)
    assert abs(l_cb - lref.item()) <= 1e-2 * abs(lref.item()), (l_cb, lref.item())
    # the bf16 passes are equally close to the fp32 gradient (both round the same operands)
    assert rel(g_cb, gref) <= 1.1 * rel(g_nc, gref) + 1e-3, (rel(g_cb, gref), rel(g_nc, gref))
    assert cos(g_cb, gref) > 0.99
