"""backward_D's stacked pass (Pix2PixModel.d_batch: D run once on the fake and real batches stacked
into 2N images) against the reference's two N-image passes (DSGAN/models/pix2pix_model.py:141-162),
at the configs[1] shape (256^2, batch 16) and the configs[4] shape (512^2, batch 8), in fp32, bf16 and
fp16.

D is per sample (InstanceNorm per plane, no BatchNorm), so the logits must be the same bits; the
weight-grads sum over the batch in another order (split-K plans follow the batch), so they agree to
fp32 reassociation, plus in the 16-bit modes one operand rounding of the split data-grads; the biases
ahead of an InstanceNorm have an analytic gradient of 0 and are held to a floor set by the weight
gradient of their layer.
"""
import random

import pytest
import torch

from oracle import dsgan_cpu as O
from oracle.recipe import make_params, synth_pair

pytestmark = pytest.mark.gpu

# per-tensor relative bars of the D weight-grads, stacked vs two-pass (measured: fp32 <= 7e-7;
# bf16 <= 1e-4 and fp16 <= 6e-5 at 512^2, where the stride-1 data-grad split count follows the batch)
REL = {"fp32": 2e-6, "bf16": 5e-4, "fp16": 5e-4}
IN_BIAS = ("model.2.bias", "model.5.bias", "model.8.bias")   # conv biases ahead of an InstanceNorm


def _model(prec, batch):
    import dsgan_hip
    from options.train_options import default_train_opt
    from models import create_model
    dsgan_hip.require_gpu()
    random.seed(20)
    torch.manual_seed(20)
    m = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision=prec, batchSize=batch))
    with torch.no_grad():
        for net, pr in ((m.netG, make_params(O.g_param_spec(), "ref", 1000)),
                        (m.netD, make_params(O.d_param_spec(), "ref", 5000)),
                        (m.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    return m


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("size,batch", [(256, 16), (512, 8)])
def test_stacked_d_equals_two_pass(prec, size, batch):
    m = _model(prec, batch)
    A, B = synth_pair(batch, size, seed=51)
    m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * batch, "B_paths": [""] * batch})
    m.forward()
    s0 = m.scaler_D.state.clone() if m.scaler_D is not None else None
    res = {}
    for form in (False, True):
        m.d_batch = form
        m.set_requires_grad(m.netD, True)
        m.optimizer_D.zero_grad()
        m.backward_D()
        if m.scaler_D is not None:
            m.scaler_D.check(m.flatD.grad)
        torch.cuda.synchronize()
        res[form] = dict(pf=m.pred_fake.detach().clone(), pr=m.pred_real.detach().clone(),
                         L=(m.loss_D_fake.item(), m.loss_D_real.item(), m.loss_D.item()),
                         g={k: p.grad.detach().clone() for k, p in m.netD.named_parameters()},
                         sc=m.scaler_D.state.clone() if s0 is not None else None)
        if s0 is not None:
            m.scaler_D.state.copy_(s0)
    two, st = res[False], res[True]
    assert torch.equal(st["pf"], two["pf"]) and torch.equal(st["pr"], two["pr"])
    assert st["L"] == two["L"]
    if s0 is not None:
        assert torch.equal(st["sc"], two["sc"]), (st["sc"], two["sc"])
        assert st["sc"][1].item() == 0.0   # no skipped step
    msg = []
    for k, g2 in two["g"].items():
        gs = st["g"][k]
        assert torch.isfinite(gs).all(), k
        if k in IN_BIAS:
            gw = two["g"][k.replace("bias", "weight")].double().norm().item()
            ok = (gs.double() - g2.double()).norm().item() <= 2e-6 * gw
        else:
            ok = _rel(gs, g2) <= REL[prec]
        msg.append("%s %.2e" % (k, _rel(gs, g2)))
        assert ok, (k, msg)
    print("%s %d^2 b%d: %s" % (prec, size, batch, ", ".join(msg)))


@pytest.mark.timeout(900)
def test_c5_fp16_trajectory_stacked_vs_two_pass():
    """configs[4] (fp16, 512^2, batch 8) from the reference init, 6 steps with each form of backward_D:
    no step of either network skipped by the loss scaler in either run (the round-5 stacked run
    skipped G's step 4 on the SSIM backward's NaN: tests/test_ops_gpu.py::
    test_ssim_bwd_finite_where_covariance_crosses_minus_c2) and the two runs' fake_B MS-SSIM against the
    target within 1e-4 of each other (the north-star bar vs the reference is 1e-3)."""
    outs = []
    for form in (False, True):
        m = _model("fp16", 8)
        m.d_batch = form
        for i in range(6):
            A, B = synth_pair(8, 512, seed=100 + i)
            m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * 8, "B_paths": [""] * 8})
            m.optimize_parameters()
        torch.cuda.synchronize()
        rep = m.nonfinite_report()
        outs.append((rep, m.scaler_G.get_scale(), m.scaler_D.get_scale(), m.fake_B.detach().float().cpu()))
        del m
        torch.cuda.empty_cache()
    tgt = (B + 1) / 2
    ms = [O.ms_ssim((f + 1) / 2, tgt).item() for *_, f in outs]
    print("reports %s / %s, ms_ssim two-pass %.6f stacked %.6f" % (outs[0][0], outs[1][0], ms[0], ms[1]))
    for rep, sG, sD, _ in outs:
        assert rep == {"G": (0, 6), "D": (0, 6)} and sG == sD == 2.0 ** 16, (rep, sG, sD)
    assert abs(ms[0] - ms[1]) <= 1e-4, ms
