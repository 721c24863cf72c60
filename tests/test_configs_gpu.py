"""Parity at the BASELINE.json configurations themselves:

  * C2 (configs[1]): one bf16 G+D step at 256x256, batch 16, vs the fp32 oracle step on the
    same batch (DSGAN/models/pix2pix_model.py:201-217).  Bars: losses <= 2e-2 relative,
    SSIM(fake_bf16, fake_ref) >= 0.999, cosine >= 0.999 of the flat G and D gradients.
  * C4 shape (configs[3], per GPU): one bf16 step at 256x256, batch 32, with the opt-in MS-SSIM
    loss (--ssim_loss ms_ssim, DSGAN/MS_SSIM.py:153-225) vs the fp32 oracle step walked in chunks
    of 8 (OracleStep.step_chunked): the C2 bars on losses, fake_B and the flat G / D gradients.
  * C5 (configs[4], per GPU) as named: one fp16 step at 512x512, batch 8 (fp16 MFMA operands and
    16-bit storage, fp32 accumulation, device loss scaling) vs the fp32 oracle step on the same
    batch (OracleStep.step_chunked: the 512^2 autograd graph is walked 2 samples at a time), with
    the C2 bars, finite gradients and no overflow-skipped step; plus the same shape in bf16 (the
    input-only terms).
All at the reference's N(0, 0.02) init ("ref" weight recipe), pool_size 0.
"""
import random

import pytest
import torch

from oracle import dsgan_cpu as O
from oracle.recipe import make_params, synth_pair

pytestmark = pytest.mark.gpu


def _model(precision, batch, recipe="ref", **over):
    import dsgan_hip
    from options.train_options import default_train_opt
    from models import create_model
    dsgan_hip.require_gpu()
    random.seed(20)
    torch.manual_seed(20)
    m = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision=precision, batchSize=batch, **over))
    gp = make_params(O.g_param_spec(), recipe, 1000)
    dp = make_params(O.d_param_spec(), recipe, 5000)
    with torch.no_grad():
        for net, pr in ((m.netG, gp), (m.netD, dp), (m.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    return m, gp, dp


def _vp():
    return make_params(O.vgg_param_spec(False), "vgg", 7000)


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return (a @ b / (a.norm() * b.norm())).item()


def _img_ssim(a, b):
    lo, hi = b.min(), b.max()
    return O.ssim((a - lo) / (hi - lo), (b - lo) / (hi - lo)).item()


def _losses(m):
    return dict(G_GAN=float(m.loss_G_GAN), G_L1=float(m.loss_G_L1), D_real=float(m.loss_D_real),
                D_fake=float(m.loss_D_fake), vgg=float(m.loss_vgg), ssim=float(m.loss_ssim))


@pytest.mark.timeout(1200)
def test_c2_bf16_step_b16_vs_oracle():
    torch.set_num_threads(16)
    m, gp, dp = _model("bf16", 16)
    A, B = synth_pair(16, 256, seed=21)
    m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * 16, "B_paths": [""] * 16})
    m.optimize_parameters()
    torch.cuda.synchronize()
    got = _losses(m)
    gG = torch.cat([p.grad.detach().flatten() for p in m.netG.parameters()]).cpu()
    gD = torch.cat([p.grad.detach().flatten() for p in m.netD.parameters()]).cpu()
    fake = m.fake_B.detach().cpu()
    del m
    torch.cuda.empty_cache()
    st = O.OracleStep(gp, dp, _vp(), pool_size=0)
    L = st.step(A, B)
    rG = torch.cat([v.grad.flatten() for v in st.gp.values()])
    rD = torch.cat([v.grad.flatten() for v in st.dp.values()])
    msg = {k: (v, L[k]) for k, v in got.items()}
    for k, v in got.items():
        assert abs(v - L[k]) <= 2e-2 * abs(L[k]) + 1e-4, msg
    s = _img_ssim(fake, st.fake_B)
    cg, cd = _cos(gG, rG), _cos(gD, rD)
    print("C2: ssim(fake) %.6f  cos(gG) %.5f  cos(gD) %.5f  losses %s" % (s, cg, cd, msg))
    assert s >= 0.999, s
    assert cg >= 0.999 and cd >= 0.999, (cg, cd)


def _oracle_input_terms(gp, dp, vp, A, B, chunk, ssim_kind="ssim"):
    """Batch means of the step terms that only depend on the inputs and the initial weights,
    accumulated chunk by chunk (each is a mean over samples, so chunk means average exactly)."""
    acc = dict(G_L1=0.0, vgg=0.0, D_real=0.0, D_fake=0.0, ssim=0.0)
    fakes = []
    n = A.shape[0]
    with torch.no_grad():
        for i in range(0, n, chunk):
            a, b = A[i:i + chunk], B[i:i + chunk]
            w = a.shape[0] / n
            f = O.g_fwd(gp, a)
            fakes.append(f)
            acc["D_fake"] += w * O.bce_logits(O.d_fwd(dp, torch.cat((a, f), 1)), 0.0).item()
            acc["D_real"] += w * O.bce_logits(O.d_fwd(dp, torch.cat((a, b), 1)), 1.0).item()
            acc["G_L1"] += w * torch.mean(torch.abs(f - b)).item()
            fr, ff = O.vgg_fwd(vp, b), O.vgg_fwd(vp, f)
            acc["vgg"] += w * sum(torch.mean(torch.abs(x - y)).item() for x, y in zip(ff[:4], fr[:4]))
            fn = O.ms_ssim if ssim_kind == "ms_ssim" else O.ssim
            acc["ssim"] += w * (1 - fn((b + 1) / 2, (f + 1) / 2).item())
    return acc, torch.cat(fakes)


def _check_input_terms(m, gp, dp, A, B, chunk, ssim_kind):
    got = _losses(m)
    fake = m.fake_B.detach().cpu()
    peak = torch.cuda.max_memory_allocated() / 2 ** 30
    ref, rfake = _oracle_input_terms(gp, dp, _vp(), A, B, chunk, ssim_kind)
    msg = {k: (got[k], v) for k, v in ref.items()}
    for k, v in ref.items():
        assert abs(got[k] - v) <= 2e-2 * abs(v) + 1e-4, msg
    s = _img_ssim(fake, rfake)
    print("peak HBM %.1f GiB, ssim(fake) %.6f, %s" % (peak, s, msg))
    assert s >= 0.999, s
    for k in ("G_GAN", "G_L1", "vgg", "ssim", "D_real", "D_fake"):
        assert torch.isfinite(torch.tensor(got[k])), k
    for net in (m.netG, m.netD):
        for p in net.parameters():
            assert torch.isfinite(p).all()


@pytest.mark.timeout(1500)
def test_c4_bf16_step_b32_msssim():
    """configs[3] per GPU: one bf16 step at 256x256, batch 32, with the opt-in MS-SSIM loss
    (DSGAN/MS_SSIM.py:153-225 in place of pix2pix_model.py:195) vs the fp32 oracle step on the same
    batch, walked 8 samples at a time (OracleStep.step_chunked; every term is a batch mean of
    per-image values -- ms_ssim included, :222-225 -- except TV, a batch sum): the C2 bars on the
    losses, the generated batch and the flat G and D gradients, which carry the MS-SSIM backward
    through the whole generator."""
    torch.set_num_threads(16)
    torch.cuda.reset_peak_memory_stats()
    m, gp, dp = _model("bf16", 32, ssim_loss="ms_ssim")
    A, B = synth_pair(32, 256, seed=41)
    m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * 32, "B_paths": [""] * 32})
    m.optimize_parameters()
    torch.cuda.synchronize()
    got = _losses(m)
    gG = torch.cat([p.grad.detach().flatten() for p in m.netG.parameters()]).cpu()
    gD = torch.cat([p.grad.detach().flatten() for p in m.netD.parameters()]).cpu()
    fake = m.fake_B.detach().cpu()
    finite = all(bool(torch.isfinite(p).all()) for net in (m.netG, m.netD) for p in net.parameters())
    skipped = (m.scaler_G.skipped_last(), m.scaler_D.skipped_last()) if m.scaler_G is not None else (False, False)
    peak = torch.cuda.max_memory_allocated() / 2 ** 30
    del m
    torch.cuda.empty_cache()
    assert finite and skipped == (False, False) and torch.isfinite(gG).all() and torch.isfinite(gD).all()
    st = O.OracleStep(gp, dp, _vp(), pool_size=0, ssim_kind="ms_ssim")
    L = st.step_chunked(A, B, 8)
    rG = torch.cat([v.grad.flatten() for v in st.gp.values()])
    rD = torch.cat([v.grad.flatten() for v in st.dp.values()])
    msg = {k: (v, L[k]) for k, v in got.items()}
    s = _img_ssim(fake, st.fake_B)
    cg, cd = _cos(gG, rG), _cos(gD, rD)
    print("C4: peak HBM %.1f GiB, ssim(fake) %.6f  cos(gG) %.5f  cos(gD) %.5f  losses %s" % (peak, s, cg, cd, msg))
    for k, v in got.items():
        assert abs(v - L[k]) <= 2e-2 * abs(L[k]) + 1e-4, msg
    assert s >= 0.999, s
    assert cg >= 0.999 and cd >= 0.999, (cg, cd)


@pytest.mark.timeout(1200)
def test_c5_bf16_step_512_b8():
    torch.set_num_threads(16)
    torch.cuda.reset_peak_memory_stats()
    m, gp, dp = _model("bf16", 8)
    A, B = synth_pair(8, 512, seed=51)
    m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * 8, "B_paths": [""] * 8})
    m.optimize_parameters()
    torch.cuda.synchronize()
    _check_input_terms(m, gp, dp, A, B, 2, "ssim")


@pytest.mark.timeout(1500)
def test_c5_fp16_step_512_b8_vs_oracle():
    torch.set_num_threads(16)
    torch.cuda.reset_peak_memory_stats()
    m, gp, dp = _model("fp16", 8)
    A, B = synth_pair(8, 512, seed=51)
    m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * 8, "B_paths": [""] * 8})
    m.optimize_parameters()
    torch.cuda.synchronize()
    got = _losses(m)
    skipped = (m.scaler_G.skipped_last(), m.scaler_D.skipped_last())
    gG = torch.cat([p.grad.detach().flatten() for p in m.netG.parameters()]).cpu()
    gD = torch.cat([p.grad.detach().flatten() for p in m.netD.parameters()]).cpu()
    fake = m.fake_B.detach().cpu()
    finite_params = all(bool(torch.isfinite(p).all()) for net in (m.netG, m.netD) for p in net.parameters())
    peak = torch.cuda.max_memory_allocated() / 2 ** 30
    del m
    torch.cuda.empty_cache()
    assert skipped == (False, False), skipped
    assert torch.isfinite(gG).all() and torch.isfinite(gD).all() and finite_params
    st = O.OracleStep(gp, dp, _vp(), pool_size=0)
    L = st.step_chunked(A, B, 2)
    rG = torch.cat([v.grad.flatten() for v in st.gp.values()])
    rD = torch.cat([v.grad.flatten() for v in st.dp.values()])
    msg = {k: (v, L[k]) for k, v in got.items()}
    s = _img_ssim(fake, st.fake_B)
    cg, cd = _cos(gG, rG), _cos(gD, rD)   # (the flat grads hold the loss-scaled gradient: cosine is scale-free)
    print("C5 fp16: peak HBM %.1f GiB, ssim(fake) %.6f  cos(gG) %.5f  cos(gD) %.5f  losses %s" % (peak, s, cg, cd, msg))
    for k, v in got.items():
        assert abs(v - L[k]) <= 2e-2 * abs(L[k]) + 1e-4, msg
    assert s >= 0.999, s
    assert cg >= 0.999 and cd >= 0.999, (cg, cd)
