"""Command-line options (DSGAN/options/base_options.py:8-141) -- same flag names, defaults and
``parse(dataset_path, path)`` signature, plus two build flags:

  --precision {fp32,bf16}   MFMA operand precision of the HIP contractions (fp32 = parity mode)
  --vgg_weights PATH        local VGG16 weights (the reference downloads ImageNet weights)

The untyped loss-weight flags of the reference (quirk q1: ``--w_gan 0.1`` on the CLI becomes a
str and crashes the reference) are kept as declared; the model casts them to numbers.
Under ``torchrun`` each rank uses ``cuda:LOCAL_RANK`` (one process per GPU).
"""
import argparse
import os

import torch

import models


class BaseOptions:
    def __init__(self):
        self.initialized = False

    def initialize(self, parser):
        parser.add_argument("--dataroot", type=str, default="/root/dataset/256x256",
                            help="path to images (should have subfolders trainA, trainB, valA, valB, etc)")
        parser.add_argument("--batchSize", type=int, default=1, help="input batch size")
        parser.add_argument("--loadSize_w", type=int, default=256, help="scale images to this size")
        parser.add_argument("--fineSize_w", type=int, default=256, help="then crop to this size")
        parser.add_argument("--loadSize_h", type=int, default=256, help="scale images to this size")
        parser.add_argument("--fineSize_h", type=int, default=256, help="then crop to this size")
        parser.add_argument("--input_nc", type=int, default=3, help="# of input image channels")
        parser.add_argument("--output_nc", type=int, default=3, help="# of output image channels")
        parser.add_argument("--ngf", type=int, default=32, help="# of gen filters in first conv layer")
        parser.add_argument("--ndf", type=int, default=32, help="# of discrim filters in first conv layer")
        parser.add_argument("--which_model_netD", type=str, default="basic", help="selects model to use for netD")
        parser.add_argument("--which_model_netG", type=str, default="MixConvNeXtML", help="selects model to use for netG")
        parser.add_argument("--n_layers_D", type=int, default=3, help="only used if which_model_netD==n_layers")
        parser.add_argument("--gpu_ids", type=str, default="0", help="gpu ids: e.g. 0  0,1,2, 0,2. use -1 for CPU")
        parser.add_argument("--name", type=str, default="experiment_name",
                            help="name of the experiment. It decides where to store samples and models")
        parser.add_argument("--dataset_mode", type=str, default="aligned",
                            help="chooses how datasets are loaded. [unaligned | aligned | single]")
        parser.add_argument("--model", type=str, default="pix2pix",
                            help="chooses which model to use. cycle_gan, pix2pix, test,d3")
        parser.add_argument("--which_direction", type=str, default="AtoB", help="AtoB or BtoA")
        parser.add_argument("--nThreads", default=4, type=int, help="# threads for loading data")
        parser.add_argument("--checkpoints_dir", type=str, default="./checkpoints/", help="models are saved here")
        parser.add_argument("--norm", type=str, default="instance",
                            help="instance normalization or batch normalization")
        parser.add_argument("--serial_batches", action="store_true",
                            help="if true, takes images in order to make batches, otherwise takes them randomly")
        parser.add_argument("--display_winsize", type=int, default=256, help="display window size")
        parser.add_argument("--display_id", type=int, default=1, help="window id of the web display")
        parser.add_argument("--display_server", type=str, default="http://localhost",
                            help="visdom server of the web display")
        parser.add_argument("--display_port", type=int, default=8097, help="visdom port of the web display")
        parser.add_argument("--no_dropout", action="store_true", help="no dropout for the generator")
        parser.add_argument("--max_dataset_size", type=int, default=float("inf"),
                            help="Maximum number of samples allowed per dataset.")
        parser.add_argument("--resize_or_crop", type=str, default="resize_and_crop",
                            help="scaling and cropping of images at load time [resize_and_crop|crop|scale_width|scale_width_and_crop]")
        parser.add_argument("--no_flip", action="store_true",
                            help="if specified, do not flip the images for data augmentation")
        parser.add_argument("--init_type", type=str, default="normal",
                            help="network initialization [normal|xavier|kaiming|orthogonal]")
        parser.add_argument("--verbose", action="store_true", help="if specified, print more debugging information")
        parser.add_argument("--suffix", default="", type=str,
                            help="customized suffix: opt.name = opt.name + suffix")
        parser.add_argument("--use_GAN", default=1, help="1 is use gan")
        parser.add_argument("--w_gan", default=0.01, help="weight of the gan loss")
        parser.add_argument("--w_vgg", default=1, help="weight of the vgg loss")
        parser.add_argument("--w_tv", default=1, help="weight of the tv loss")
        parser.add_argument("--w_ss", default=1.25, help="weight of the ms-ssim loss")
        parser.add_argument("--use_condition", default=1, help="1 means add condition in discriminator")
        # ---- MI355X build flags ----
        parser.add_argument("--precision", type=str, default="fp32", choices=["fp32", "bf16", "fp16"],
                            help="operand precision of the MFMA contractions (accumulation is fp32)")
        parser.add_argument("--vgg_weights", type=str, default="",
                            help="local VGG16 weights (torchvision features.* or Vgg16 state dict)")
        self.initialized = True
        return parser

    def gather_options(self, args=None):
        if not self.initialized:
            parser = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
            parser = self.initialize(parser)
        opt, _ = parser.parse_known_args(args)
        model_option_setter = models.get_option_setter(opt.model)
        parser = model_option_setter(parser, self.isTrain)
        self.parser = parser
        return parser.parse_args(args)

    def print_options(self, opt):
        message = "----------------- Options ---------------\n"
        for k, v in sorted(vars(opt).items()):
            comment = ""
            default = self.parser.get_default(k)
            if v != default:
                comment = "\t[default: %s]" % str(default)
            message += "{:>25}: {:<30}{}\n".format(str(k), str(v), comment)
        message += "----------------- End -------------------"
        print(message)
        expr_dir = os.path.join(opt.checkpoints_dir, opt.name)
        os.makedirs(expr_dir, exist_ok=True)
        with open(os.path.join(expr_dir, "opt.txt"), "wt") as opt_file:
            opt_file.write(message)
            opt_file.write("\n")

    def parse(self, dataset_path, path, args=None):
        opt = self.gather_options(args)
        opt.isTrain = self.isTrain
        opt.checkpoints_dir = os.path.join(path, "checkpoints")
        opt.dataroot = dataset_path
        if opt.suffix:
            opt.name = opt.name + ("_" + opt.suffix.format(**vars(opt)))
        self.print_options(opt)
        opt.gpu_ids = [int(s) for s in str(opt.gpu_ids).split(",") if int(s) >= 0]
        if "LOCAL_RANK" in os.environ and opt.gpu_ids:
            opt.gpu_ids = [int(os.environ["LOCAL_RANK"])]
        if len(opt.gpu_ids) > 0:
            torch.cuda.set_device(opt.gpu_ids[0])
        self.opt = opt
        return self.opt
