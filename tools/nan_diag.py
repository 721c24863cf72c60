"""GPU-only replay of bench.py's quality leg (B=16, 256^2, reference init, bf16, 10 steps): per-step
losses and the first non-finite value, under toggles of the recent step changes."""
import os, sys, random
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
import dsgan_hip
from dsgan_hip import functional as HF
from oracle import dsgan_cpu as O
from oracle.recipe import make_params, synth_pair
from options.train_options import default_train_opt
from models import create_model
import models.pix2pix_model as PM

dsgan_hip.require_gpu()
arms = sys.argv[1:] or ["all", "no_losssum"]
orig_fusable = PM._fusable
for arm in arms:
    PM._fusable = (lambda *a: False) if arm == "no_losssum" else orig_fusable
    HF.set_precision("bf16")
    random.seed(20); torch.manual_seed(20)
    model = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision="bf16", batchSize=16))
    gp = make_params(O.g_param_spec(), "ref", 1000)
    dp = make_params(O.d_param_spec(), "ref", 5000)
    with torch.no_grad():
        for net, pr in ((model.netG, gp), (model.netD, dp), (model.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
            for k, v in net.state_dict().items():
                v.copy_(pr[k])
    for i in range(int(os.environ.get("NAN_DIAG_STEPS", "10"))):
        A, B = synth_pair(16, 256, seed=100 + i)
        model.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * 16, "B_paths": [""] * 16})
        model.optimize_parameters()
        torch.cuda.synchronize()
        vals = dict(G=float(model.loss_G), D=float(model.loss_D), L1=float(model.loss_G_L1), vgg=float(model.loss_vgg),
                    ssim=float(model.loss_ssim), fake=float(model.fake_B.float().abs().max()),
                    gG=float(model.flatG.grad.abs().max()), gD=float(model.flatD.grad.abs().max()),
                    pG=float(model.flatG.data.abs().max()), pD=float(model.flatD.data.abs().max()))
        print(arm, i, " ".join("%s=%.4g" % kv for kv in vals.items()), flush=True)
    del model
    torch.cuda.empty_cache()
