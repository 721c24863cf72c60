"""The north-star parity sentence at the shape it names (missing #2): one
``optimize_parameters`` in ``--precision fp32`` at 256x256, batch 2, pool_size 0, against the
reference's own step at that shape (tests/golden/golden_v4.npz, written by
tests/golden/gen_golden_v4.py from the real reference) and, for the whole gradient vectors, the
fp64 oracle step (oracle/dsgan_cpu.py, pinned to the same golden by
tests/test_oracle.py::test_step_256_matches_reference).  Reference: DSGAN/models/pix2pix_model.py:201-217.

At 256^2 the step engages paths the 64^2 step tests never reach: the split-K planners at B = 2,
the 64K-pixel InstanceNorm planes (register / LDS-parked forms), the full-size VGG16 pyramid and
the thin G head.

Bars (the north star: "within 1e-3 relative fp32 tolerance"):
  * the nine losses: relative <= 1e-3 vs the reference's fp32 step and vs its fp64 step;
  * fake_B (a sample, its norm, probe dots), against both: relative <= 1e-3, or 3x the reference's
    own fp32 error / 8x its 1-ulp spread where those are larger (the N(0, 0.02) recipe: the
    reference's fp32 fake_B is 1.7e-3 off its own fp64 one on the probe dots);
  * gradients, per tensor (norm, probe dot, and for the fanin recipe the whole vector vs the fp64
    oracle): |g - g64| <= max(2 |g32_ref - g64_ref|, 2e-3 |g64|, 8 x the reference's own spread under
    1-ulp perturbations of its weights and input) + 1e-6 -- the bar of
    test_model_gpu.py::test_full_step_fp32_vs_oracle, with the conditioning measured on the
    reference itself;
  * post-Adam parameters (fanin recipe): element-wise equal to the fp64 oracle's to 2e-5 (lr 2e-4)
    wherever the step's sign is determined -- |g64| > 1e-6 and > 16x the tensor's RMS gradient error.
    A first Adam step is lr * sign(g), so an element whose gradient is ~0 at fp32 resolution steps
    either way; the golden's post-Adam probe dots sum over those elements too and are reported only.
"""
import numpy as np
import pytest
import torch

from oracle import dsgan_cpu as O
from oracle.recipe import make_params, synth_pair, probe

pytestmark = pytest.mark.gpu

NAMES = ["G_GAN", "G_L1", "D_real", "D_fake", "vgg", "tv", "ssim", "G", "D"]


def _model(recipe):
    import dsgan_hip
    from options.train_options import default_train_opt
    from models import create_model
    dsgan_hip.require_gpu()
    m = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision="fp32", batchSize=2))
    gp = make_params(O.g_param_spec(), recipe, 1000)
    dp = make_params(O.d_param_spec(), recipe, 5000)
    with torch.no_grad():
        for net, pr in ((m.netG, gp), (m.netD, dp), (m.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    return m, gp, dp


def _losses(m):
    return np.array([m.loss_G_GAN.item(), m.loss_G_L1.item(), m.loss_D_real.item(), m.loss_D_fake.item(),
                     m.loss_vgg.item(), m.tv_loss.item(), m.loss_ssim.item(), m.loss_G.item(), m.loss_D.item()])


@pytest.mark.parametrize("recipe", ["fanin", "ref"])
def test_full_step_fp32_256_vs_reference(golden_v4, recipe):
    g = golden_v4
    pre, pre64, spr = "S4_%s_f32_" % recipe, "S4_%s_f64_" % recipe, "S4_%s_spread_" % recipe
    m, gp, dp = _model(recipe)
    A, B = synth_pair(2, 256, seed=int(g["S4_input_seed"]))
    before = {nm: [p.detach().double().cpu().flatten() for p in net.parameters()] for net, nm in ((m.netG, "G"), (m.netD, "D"))}
    m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": ["a"] * 2, "B_paths": ["b"] * 2})
    m.optimize_parameters()
    torch.cuda.synchronize()
    report = []

    # losses
    got = _losses(m)
    for ref_key in (pre, pre64):
        ref = g[ref_key + "losses"]
        r = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-6)
        report.append("losses vs %s: max rel %.2e" % (ref_key, r.max()))
        assert (r <= 1e-3).all(), (ref_key, dict(zip(NAMES, r)))
    # fake_B
    fake = m.fake_B.detach().double().cpu()
    sub = fake[:, :, ::8, ::8].numpy()
    pd = np.array([float(probe(fake.numel(), 70000 + j) @ fake.flatten()) for j in range(4)])

    def fake_err(key):   # (sample, norm, probe-dot) relative errors of one fake_B against the golden's
        s_, nrm = g[key + "fake_sub"].astype(np.float64), float(g[key + "fake_norm"])
        return np.array([np.linalg.norm(sub - s_) / np.linalg.norm(s_), abs(float(fake.norm()) - nrm) / nrm,
                         np.abs(pd - g[key + "fake_pdot"]).max() / nrm])

    # the reference's own fp32 error on each measure (its fp32 fake_B against its fp64 one): 1e-6 in the
    # fanin recipe; in the N(0, 0.02) recipe 7.6e-4 / 1.7e-3 on the sample / probe dots, above the
    # north star's 1e-3 -- there the bar is that error (x3) or the 1-ulp spread (x8)
    own = np.array([np.linalg.norm(g[pre + "fake_sub"].astype(np.float64) - g[pre64 + "fake_sub"])
                    / np.linalg.norm(g[pre64 + "fake_sub"].astype(np.float64)),
                    abs(float(g[pre + "fake_norm"]) - float(g[pre64 + "fake_norm"])) / float(g[pre64 + "fake_norm"]),
                    np.abs(g[pre + "fake_pdot"] - g[pre64 + "fake_pdot"]).max() / float(g[pre64 + "fake_norm"])])
    fbar = np.maximum(np.maximum(1e-3, 3 * own), 8 * float(g[spr + "fake"]))
    for ref_key in (pre, pre64):
        e = fake_err(ref_key)
        report.append("fake_B vs %s: sample %.2e norm %.2e probe %.2e (bar %.1e)" % ((ref_key,) + tuple(e) + (fbar.max(),)))
        assert (e <= fbar).all(), (ref_key, e, fbar)

    # gradients (norm and probe dot per tensor) and post-Adam deltas, against the reference
    worst = {}
    for net, nm in ((m.netG, "G"), (m.netD, "D")):
        d32, d64, n32, n64 = (g[pre + nm + "_gdot"], g[pre64 + nm + "_gdot"], g[pre + nm + "_gnorm"],
                              g[pre64 + nm + "_gnorm"])
        u32, u64 = g[pre + nm + "_upd"], g[pre64 + nm + "_upd"]
        sv, sd, su = g[spr + nm + "_gvec"], g[spr + nm + "_gdot"], g[spr + nm + "_upd"]
        for i, (k, p) in enumerate(net.named_parameters()):
            gr = p.grad.detach().double().cpu().flatten()
            pr = probe(gr.numel(), 90000 + i)
            bar = max(2 * abs(d32[i] - d64[i]), 2 * abs(n32[i] - n64[i]), 2e-3 * n64[i], 8 * sv[i], 8 * sd[i]) + 1e-6
            e = max(abs(float(gr @ pr) - d64[i]), abs(float(gr.norm()) - n64[i]))
            worst[nm + " grad"] = max(worst.get(nm + " grad", 0.0), e / bar)
            assert e <= bar, (nm, k, e, bar, d64[i], n64[i])
            # post-Adam delta vs the reference's, reported: a first Adam step is lr * sign(g), so an
            # element whose gradient is ~0 at fp32 resolution may step either way (the element-wise
            # check against the fp64 oracle below excludes those; the golden holds probe dots only)
            upd = float((p.detach().double().cpu().flatten() - before[nm][i]) @ pr)
            ubar = max(3 * abs(u32[i] - u64[i]), 8 * su[i], 1e-3 * abs(u64[i])) + 1e-7
            worst[nm + " upd (reported)"] = max(worst.get(nm + " upd (reported)", 0.0), abs(upd - u64[i]) / ubar)
    report.append("worst error / bar: " + ", ".join("%s %.2f" % kv for kv in sorted(worst.items())))

    # whole gradient vectors against the fp64 oracle (fanin: the reference's gradients are
    # well-conditioned there; in the N(0, 0.02) recipe they are only determined to ~2 %)
    if recipe == "fanin":
        st = O.OracleStep(type(gp)((k, v.double()) for k, v in gp.items()),
                          type(dp)((k, v.double()) for k, v in dp.items()),
                          make_params(O.vgg_param_spec(False), "vgg", 7000, torch.float64), pool_size=0)
        st.step(A.double(), B.double())
        L = st.losses
        o = np.array([L[k] for k in NAMES])
        assert (np.abs(got - o) <= 1e-3 * np.abs(o)).all()
        wv, nu = 0.0, 0
        w0 = {"G": {k: v.double() for k, v in gp.items()}, "D": {k: v.double() for k, v in dp.items()}}
        for net, nm, ps in ((m.netG, "G", st.gp), (m.netD, "D", st.dp)):
            d32, d64 = g[pre + nm + "_gdot"], g[pre64 + nm + "_gdot"]
            n64, sv = g[pre64 + nm + "_gnorm"], g[spr + nm + "_gvec"]
            for i, ((k, p), q) in enumerate(zip(net.named_parameters(), ps.values())):
                gd = p.grad.detach().double().cpu()
                err = (gd - q.grad).norm().item()
                bar = max(2 * abs(d32[i] - d64[i]), 2e-3 * n64[i], 8 * sv[i]) + 1e-6
                wv = max(wv, err / bar)
                assert err <= bar, (nm, k, err, bar)
                # post-Adam parameters, element-wise, where the step's sign is determined: |g64| well
                # above Adam's eps and 16x above this tensor's RMS gradient error (bounded just above)
                big = q.grad.abs() > max(1e-6, 16 * err / max(1, gd.numel()) ** 0.5)
                if big.any():
                    du = (p.detach().double().cpu().flatten() - before[nm][i])[big.flatten()]
                    dq = (q.detach() - w0[nm][k]).flatten()[big.flatten()]
                    nu = max(nu, int(big.sum()))
                    assert (du - dq).abs().max().item() < 2e-5, (nm, k, (du - dq).abs().max().item())
        report.append("whole-vector grads vs fp64 oracle: worst error / bar %.2f; post-Adam deltas equal the "
                      "oracle's to 2e-5 (lr 2e-4) on the determined elements (%d in the largest tensor)" % (wv, nu))
    print("\n[256^2 fp32 step, %s] " % recipe + "; ".join(report))
