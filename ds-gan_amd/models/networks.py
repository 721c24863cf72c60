"""Network factory, init, scheduler, GAN loss and the PatchGAN D (DSGAN/models/networks.py).

Keeps the reference's string-dispatch surface (``define_G`` / ``define_D``, unknown names raise
``NotImplementedError``) for the networks on the DS-GAN path: ``MixConvNeXtML`` and the
``basic`` / ``n_layers`` PatchGAN.  Other reference generators are out of scope (SURVEY.md §2,
row 6x) and raise the reference's own error.
"""
import functools

import torch
import torch.nn as nn
from torch.nn import init
from torch.optim import lr_scheduler

from dsgan_hip import functional as HF
from .mixconvnext import MixConvNeXtML


def get_norm_layer(norm_type="instance"):
    """DSGAN/models/networks.py:21-30."""
    if norm_type == "batch":
        return functools.partial(nn.BatchNorm2d, affine=True, track_running_stats=True)
    if norm_type == "instance":
        return functools.partial(nn.InstanceNorm2d, affine=False, track_running_stats=False)
    if norm_type == "none":
        return None
    raise NotImplementedError("normalization layer [%s] is not found" % norm_type)


def get_scheduler(optimizer, opt):
    """DSGAN/models/networks.py:33-46 (lambda rule kept verbatim in behaviour, quirk q4)."""
    if opt.lr_policy == "lambda":
        def lambda_rule(epoch):
            return 1.0 - max(0, epoch + 1 + opt.epoch_count - opt.niter) / float(opt.niter_decay + 1)
        return lr_scheduler.LambdaLR(optimizer, lr_lambda=lambda_rule)
    if opt.lr_policy == "step":
        return lr_scheduler.StepLR(optimizer, step_size=opt.lr_decay_iters, gamma=0.1)
    if opt.lr_policy == "plateau":
        return lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=0.2, threshold=0.01, patience=5)
    return NotImplementedError("learning rate policy [%s] is not implemented", opt.lr_policy)


def init_weights(net, init_type="normal", gain=0.02):
    """DSGAN/models/networks.py:49-70: Conv*/Linear weights ~ N(0, gain) (or xavier/kaiming/
    orthogonal), biases 0, applied post-order with ``net.apply``."""
    def init_func(m):
        classname = m.__class__.__name__
        if hasattr(m, "weight") and (classname.find("Conv") != -1 or classname.find("Linear") != -1):
            if init_type == "normal":
                init.normal_(m.weight.data, 0.0, gain)
            elif init_type == "xavier":
                init.xavier_normal_(m.weight.data, gain=gain)
            elif init_type == "kaiming":
                init.kaiming_normal_(m.weight.data, a=0, mode="fan_in")
            elif init_type == "orthogonal":
                init.orthogonal_(m.weight.data, gain=gain)
            else:
                raise NotImplementedError("initialization method [%s] is not implemented" % init_type)
            if hasattr(m, "bias") and m.bias is not None:
                init.constant_(m.bias.data, 0.0)
        elif classname.find("BatchNorm2d") != -1:
            init.normal_(m.weight.data, 1.0, gain)
            init.constant_(m.bias.data, 0.0)

    print("initialize network with %s" % init_type)
    net.apply(init_func)


def init_net(net, init_type="normal", gpu_ids=()):
    """DSGAN/models/networks.py:73-79, minus ``nn.DataParallel``: the build runs one process
    per GPU (torch.distributed over RCCL), so the net is moved to this rank's device only.

    The weights are drawn on the CPU generator BEFORE the move, i.e. exactly the reference's
    ``gpu_ids=[]`` init (module construction and the post-order N(0, 0.02) draws consume the
    global CPU RNG in the same order; pinned by tests/golden/golden_v2.npz INIT_*).  (The
    reference with GPUs draws from the CUDA generator after ``net.to``, which no CPU run can pin;
    every rank of a multi-GPU run draws the same values, and rank 0's are broadcast anyway.)"""
    init_weights(net, init_type)
    if len(gpu_ids) > 0:
        assert torch.cuda.is_available(), "gpu_ids given but no ROCm GPU is visible"
        net.to(torch.device("cuda", gpu_ids[0]))
    return net


def define_G(input_nc, output_nc, ngf, which_model_netG, norm="batch", use_dropout=False,
             init_type="normal", gpu_ids=()):
    """DSGAN/models/networks.py:81-113."""
    if which_model_netG == "MixConvNeXtML":
        netG = MixConvNeXtML()
    else:
        raise NotImplementedError("Generator model name [%s] is not recognized" % which_model_netG)
    return init_net(netG, init_type, gpu_ids)


def define_D(input_nc, ndf, which_model_netD, n_layers_D=3, norm="batch", use_sigmoid=False,
             init_type="normal", gpu_ids=()):
    """DSGAN/models/networks.py:115-131.  The PatchGAN runs InstanceNorm (affine=False, the
    reference default ``--norm instance``) fused into its conv kernels; ``--norm batch`` (affine
    BatchNorm2d with running stats) and ``none`` are not on the DS-GAN path and raise instead of
    silently training a different discriminator."""
    if norm != "instance":
        raise NotImplementedError("define_D: norm [%s] is not supported by the MI355X PatchGAN "
                                  "(instance only, the reference default)" % norm)
    norm_layer = get_norm_layer(norm_type=norm)
    if which_model_netD == "basic":
        netD = NLayerDiscriminator(input_nc, ndf, n_layers=3, norm_layer=norm_layer, use_sigmoid=use_sigmoid)
    elif which_model_netD == "n_layers":
        netD = NLayerDiscriminator(input_nc, ndf, n_layers_D, norm_layer=norm_layer, use_sigmoid=use_sigmoid)
    else:
        raise NotImplementedError("Discriminator model name [%s] is not recognized" % which_model_netD)
    return init_net(netD, init_type, gpu_ids)


class GANLoss(nn.Module):
    """DSGAN/models/networks.py:143-163.  use_lsgan=False (the default, quirk q3) is
    BCEWithLogits against a constant label, computed by the fused HIP reduction."""

    def __init__(self, use_lsgan=True, target_real_label=1.0, target_fake_label=0.0):
        super().__init__()
        self.register_buffer("real_label", torch.tensor(target_real_label))
        self.register_buffer("fake_label", torch.tensor(target_fake_label))
        self.use_lsgan = use_lsgan
        if use_lsgan:
            raise NotImplementedError("LSGAN (MSE) GAN loss is not on the DS-GAN path; "
                                      "the reference default is BCEWithLogits (--no_lsgan unset)")

    def __call__(self, input, target_is_real):
        return HF.bce_with_logits(input, 1.0 if target_is_real else 0.0)


class NLayerDiscriminator(nn.Module):
    """PatchGAN D, DSGAN/models/networks.py:533-579.  Same ``model.<i>`` Sequential indices as
    the reference (conv holders at 0, 2, 5, 8, 11), forward on HIP kernels: implicit-GEMM 4x4
    conv (+bias, +LeakyReLU(0.2) in the epilogue for layer 0) and InstanceNorm + LeakyReLU fused."""

    def __init__(self, input_nc, ndf=64, n_layers=3, norm_layer=nn.BatchNorm2d, use_sigmoid=False):
        super().__init__()
        if type(norm_layer) == functools.partial:
            use_bias = norm_layer.func == nn.InstanceNorm2d
        else:
            use_bias = norm_layer == nn.InstanceNorm2d
        if use_sigmoid:
            raise NotImplementedError("use_sigmoid=True is only reachable with --no_lsgan (LSGAN)")
        kw, padw = 4, 1
        seq = [nn.Conv2d(input_nc, ndf, kernel_size=kw, stride=2, padding=padw), nn.LeakyReLU(0.2, True)]
        self.plan = [(0, 2, False)]  # (index, stride, instance_norm)
        nf_mult = 1
        for n in range(1, n_layers):
            nf_prev, nf_mult = nf_mult, min(2 ** n, 8)
            self.plan.append((len(seq), 2, True))
            seq += [nn.Conv2d(ndf * nf_prev, ndf * nf_mult, kernel_size=kw, stride=2, padding=padw, bias=use_bias),
                    norm_layer(ndf * nf_mult), nn.LeakyReLU(0.2, True)]
        nf_prev, nf_mult = nf_mult, min(2 ** n_layers, 8)
        self.plan.append((len(seq), 1, True))
        seq += [nn.Conv2d(ndf * nf_prev, ndf * nf_mult, kernel_size=kw, stride=1, padding=padw, bias=use_bias),
                norm_layer(ndf * nf_mult), nn.LeakyReLU(0.2, True)]
        self.plan.append((len(seq), 1, None))
        seq += [nn.Conv2d(ndf * nf_mult, 1, kernel_size=kw, stride=1, padding=padw)]
        self.model = nn.Sequential(*seq)

    def forward(self, x):
        h = x
        for idx, stride, use_in in self.plan:
            c = self.model[idx]
            if use_in is None:      # last conv: raw logits
                h = HF.conv2d(h, c.weight, c.bias, stride=stride, pad=1)
            elif use_in:
                h = HF.instance_norm(HF.conv2d(h, c.weight, c.bias, stride=stride, pad=1), act="lrelu")
            else:
                h = HF.conv2d(h, c.weight, c.bias, stride=stride, pad=1, act="lrelu")
        return h
