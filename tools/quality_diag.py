"""Diagnostic: which sub-network's bf16 rounding moves the MS-SSIM quality metric.

Trains the CPU oracle once (fp32, reference N(0,0.02) recipe, 10 steps at 256^2, batch 2 --
the same leg as bench.py's "quality"), then the GPU model in several precision mixes from the
same weights/inputs, and prints |MS-SSIM(fake_gpu, B) - MS-SSIM(fake_ref, B)| per mix.
usage: python tools/quality_diag.py [steps]"""
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch  # noqa: E402

from oracle import dsgan_cpu as O  # noqa: E402
from oracle.recipe import make_params, synth_pair  # noqa: E402
from options.train_options import default_train_opt  # noqa: E402
from models import create_model  # noqa: E402
from dsgan_hip import functional as HF  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
batch, size = 2, 256
torch.set_num_threads(16)
gp = make_params(O.g_param_spec(), "ref", 1000)
dp = make_params(O.d_param_spec(), "ref", 5000)
vp_full = make_params(O.vgg_param_spec(True), "vgg", 7000)
data = [synth_pair(batch, size, seed=100 + i) for i in range(steps)]

t0 = time.time()
ref = O.OracleStep(gp, dp, make_params(O.vgg_param_spec(False), "vgg", 7000), pool_size=0)
for A, B in data:
    ref.step(A, B)
tgt = (data[-1][1] + 1) / 2
m_ref = O.ms_ssim((ref.fake_B + 1) / 2, tgt).item()
print("oracle fp32: ms_ssim %.6f (%.1f s)" % (m_ref, time.time() - t0), flush=True)


def pin(mod, prec):
    f = mod.forward

    def g(*a, **k):
        with HF.precision(prec):
            return f(*a, **k)
    mod.forward = g


def run(base, fp32_parts=()):
    """base "bf16-nopin": bf16 everywhere, the MidMLKA 1x1 conv included (its shipped fp32 pin off)."""
    from models.mixconvnext import MidMLKA
    label = base
    MidMLKA.conv_precision = "bf16" if base == "bf16-nopin" else "fp32"
    base = "bf16" if base == "bf16-nopin" else base
    random.seed(20)
    torch.manual_seed(20)
    model = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision=base, batchSize=batch, cuda_graph=0))
    with torch.no_grad():
        for net, pr in ((model.netG, gp), (model.netD, dp), (model.vgg, vp_full)):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    for name in fp32_parts:
        obj = model
        for a in name.split("."):
            obj = obj[int(a)] if a.isdigit() else getattr(obj, a)
        pin(obj, "fp32")
    for A, B in data:
        model.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * batch, "B_paths": [""] * batch})
        model.optimize_parameters()
    fg = model.fake_B.detach().float().cpu()
    m = O.ms_ssim((fg + 1) / 2, tgt).item()
    sim = O.ms_ssim(((fg + 1) / 2).clamp(0, 1), ((ref.fake_B + 1) / 2).clamp(0, 1)).item()
    rel = ((fg - ref.fake_B).norm() / ref.fake_B.norm()).item()
    print("%-40s delta %.6f  ms_ssim(gpu,ref) %.4f  rel-l2(fake) %.3e" % (label + " +fp32:" + ",".join(fp32_parts),
                                                                        abs(m - m_ref), sim, rel), flush=True)
    MidMLKA.conv_precision = "fp32"


MID = ("netG.local.mid32", "netG.local.mid64", "netG.local.mid128", "netG.local.mid256")
UPC = ("netG.local.upc1.1", "netG.local.upc2", "netG.local.upc3")
UPS = ("netG.local.up1", "netG.local.up2", "netG.local.up3")
# "bf16" = the shipped policy (MidMLKA 1x1 pinned to fp32); "bf16-nopin" = everything bf16
variants = [("fp32", ()), ("bf16", ()), ("bf16-nopin", ()),
            ("bf16-nopin", MID + UPC), ("bf16-nopin", MID), ("bf16-nopin", UPC), ("bf16-nopin", UPS)]
if len(sys.argv) > 2:
    variants = [("bf16", tuple(v.split(","))) for v in sys.argv[2:]]
for base, parts in variants:
    run(base, parts)
