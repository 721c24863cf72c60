"""Generate golden fixtures by importing the REAL reference (run in this container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py [/root/reference]

The reference is pure Python on PyTorch.  Its hot path imports cleanly once the
absent third-party modules that ``optimize_parameters`` never calls are stubbed
(pytorch_msssim, pytorch_ssim, skimage -- imported at
DSGAN/models/pix2pix_model.py:9,16,19) and torchvision's ``vgg16`` is replaced by
the same ``features`` layer layout (the ImageNet weights are a remote download,
DSGAN/models/vgg.py:8; fixtures use the synthetic weights of oracle/recipe.py).
Nothing here is shipped: the outputs are the .npz fixtures next to this script.
"""
import argparse
import json
import os
import random
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle.recipe import make_params, synth_pair, probe  # noqa: E402


def _vgg16_features():
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
    layers, c = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(c, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            c = v
    return nn.Sequential(*layers)


def install_stubs():
    for name in ("pytorch_msssim", "pytorch_ssim", "skimage", "skimage.metrics", "cv2"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["skimage.metrics"].peak_signal_noise_ratio = None
    sys.modules["skimage.metrics"].structural_similarity = None
    tv = types.ModuleType("torchvision")
    tv.models = types.SimpleNamespace(vgg16=lambda pretrained=False: types.SimpleNamespace(
        features=_vgg16_features()))
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tv.models


def load_sd(net, params):
    sd = net.state_dict()
    assert list(sd.keys()) == list(params.keys()), "state_dict key order mismatch"
    net.load_state_dict({k: v.to(sd[k].dtype) for k, v in params.items()})


def ref_opt(ref_dsgan, pool_size):
    """Reference defaults, read from its own parsers without parsing argv/writing files."""
    from options.base_options import BaseOptions
    from options.train_options import TrainOptions
    p = argparse.ArgumentParser()
    TrainOptions.initialize(TrainOptions(), p)
    from models.pix2pix_model import Pix2PixModel
    Pix2PixModel.modify_commandline_options(p, True)
    opt = p.parse_args([])
    opt.isTrain = True
    opt.gpu_ids = []
    opt.checkpoints_dir = "/tmp/dsgan_golden_ckpt"
    opt.pool_size = pool_size
    return opt, p


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    dsgan = os.path.join(ref, "DSGAN")
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    install_stubs()
    sys.path.insert(0, dsgan)
    import models.pix2pix_model as p2p
    from models import networks
    from models.vgg import Vgg16
    import MS_SSIM

    class Vgg16Ref(Vgg16):  # `.type(torch.cuda.FloatTensor)` at pix2pix_model.py:118 -> no-op
        def type(self, *_a, **_k):
            return self

    p2p.Vgg16 = Vgg16Ref

    opt, parser = ref_opt(dsgan, 0)
    # ---- option defaults (plugin-surface parity) ----
    defaults = {a.dest: a.default for a in parser._actions if a.dest != "help"}
    defaults = {k: (v if isinstance(v, (int, float, str, bool, type(None))) and v != float("inf")
                    else str(v)) for k, v in defaults.items()}
    with open(os.path.join(HERE, "train_option_defaults.json"), "w") as f:
        json.dump(defaults, f, indent=1, sort_keys=True)

    from oracle.dsgan_cpu import g_param_spec, d_param_spec, vgg_param_spec

    def build(dtype, recipe):
        torch.manual_seed(20)
        random.seed(20)
        m = p2p.Pix2PixModel()
        m.initialize(opt)
        gp = make_params(g_param_spec(), recipe, 1000)
        dp = make_params(d_param_spec(), recipe, 5000)
        vp = make_params(vgg_param_spec(True), "vgg", 7000)
        load_sd(m.netG, gp)
        load_sd(m.netD, dp)
        load_sd(m.vgg, vp)
        if dtype == torch.float64:
            m.netG.double(); m.netD.double(); m.vgg.double()
            m.optimizer_G = torch.optim.Adam(m.netG.parameters(), lr=opt.lr, betas=(opt.beta1, 0.999))
            m.optimizer_D = torch.optim.Adam(m.netD.parameters(), lr=opt.lr, betas=(opt.beta1, 0.999))
        return m

    out = {}
    # key inventory
    m = build(torch.float32, "ref")
    out["g_keys"] = np.array(list(m.netG.state_dict().keys()))
    out["g_shapes"] = np.array([json.dumps(list(v.shape)) for v in m.netG.state_dict().values()])
    out["d_keys"] = np.array(list(m.netD.state_dict().keys()))
    out["vgg_keys"] = np.array(list(m.vgg.state_dict().keys()))

    # ---- F1/F2: G and D forward (64x64) ----
    for recipe in ("ref", "fanin"):
        m = build(torch.float32, recipe)
        A, B = synth_pair(1, 64, seed=1)
        with torch.no_grad():
            out["F1_%s_out" % recipe] = m.netG(A).numpy()
        A2, B2 = synth_pair(2, 64, seed=2)
        with torch.no_grad():
            out["F2_%s_out" % recipe] = m.netD(torch.cat((A2, B2), 1)).numpy()
    out["F1_in"] = synth_pair(1, 64, seed=1)[0].numpy()

    # ---- F3: ssim / ms_ssim ----
    g = torch.Generator().manual_seed(3)
    X = torch.rand(2, 3, 64, 64, generator=g)
    Y = (X + 0.2 * torch.randn(2, 3, 64, 64, generator=g)).clamp(0, 1)
    out["F3_ssim"] = np.array(float(MS_SSIM.ssim(X, Y, data_range=1)))
    X2 = torch.rand(1, 3, 176, 176, generator=g)
    Y2 = (X2 + 0.2 * torch.randn(1, 3, 176, 176, generator=g)).clamp(0, 1)
    out["F3_msssim"] = np.array(float(MS_SSIM.ms_ssim(X2, Y2, data_range=1)))

    # ---- F4/F7: one optimize_parameters at 64^2, B=2, pool_size=0 ----
    loss_names = ["loss_G_GAN", "loss_G_L1", "loss_D_real", "loss_D_fake", "loss_vgg", "tv_loss",
                  "loss_ssim", "loss_G", "loss_D"]
    for recipe in ("ref", "fanin"):
        for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
            m = build(dt, recipe)
            A, B = synth_pair(2, 64, seed=4)
            m.set_input({"A": A.to(dt), "B": B.to(dt), "A_paths": ["a"] * 2, "B_paths": ["b"] * 2})
            g0 = {k: v.detach().clone() for k, v in m.netG.state_dict().items()}
            d0 = {k: v.detach().clone() for k, v in m.netD.state_dict().items()}
            m.optimize_parameters()
            pre = "F4_%s_%s_" % (recipe, tag)
            out[pre + "losses"] = np.array([float(getattr(m, n)) for n in loss_names])
            out[pre + "fake"] = m.fake_B.detach().double().numpy()
            for net, p0, nm in ((m.netG, g0, "G"), (m.netD, d0, "D")):
                norms, dots, upd = [], [], []
                for i, (k, prm) in enumerate(net.named_parameters()):
                    gr = prm.grad.detach().double().flatten()
                    pr = probe(gr.numel(), 90000 + i)
                    norms.append(float(gr.norm()))
                    dots.append(float(gr @ pr))
                    upd.append(float((prm.detach().double().flatten() - p0[k].double().flatten()) @ pr))
                out[pre + nm + "_gnorm"] = np.array(norms)
                out[pre + nm + "_gdot"] = np.array(dots)
                out[pre + nm + "_upd"] = np.array(upd)
    out["F4_loss_names"] = np.array(loss_names)

    # ---- F5: 4-iteration trajectory with a pool of 3 (pins ImagePool RNG use) ----
    opt.pool_size = 3
    m = build(torch.float32, "fanin")
    random.seed(20)
    traj = []
    for it in range(4):
        A, B = synth_pair(2, 64, seed=100 + it)
        m.set_input({"A": A, "B": B, "A_paths": ["a"] * 2, "B_paths": ["b"] * 2})
        m.optimize_parameters()
        traj.append([float(getattr(m, n)) for n in loss_names])
    out["F5_traj"] = np.array(traj)
    opt.pool_size = 0

    # ---- lambda LR multipliers (q4) ----
    opt2 = argparse.Namespace(lr_policy="lambda", epoch_count=1, niter=10, niter_decay=10)
    sgd = torch.optim.SGD([torch.zeros(1, requires_grad=True)], lr=1.0)
    sch = networks.get_scheduler(sgd, opt2)
    mults = []
    for _ in range(21):
        mults.append(sgd.param_groups[0]["lr"])
        sgd.step(); sch.step()
    out["lr_mults"] = np.array(mults)

    np.savez_compressed(os.path.join(HERE, "golden_v1.npz"), **out)
    print("wrote", os.path.join(HERE, "golden_v1.npz"))


if __name__ == "__main__":
    main()
