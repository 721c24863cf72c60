"""Frozen VGG16 perceptual feature pass (DSGAN/models/vgg.py) on HIP kernels.

Same module tree as the reference (``to_relu_1_2.0.weight`` ... ``to_relu_5_3.28.bias``), so a
torchvision ``vgg16`` ``features.*`` state dict or a reference ``Vgg16`` state dict loads.  The
reference downloads ImageNet weights (``pretrained=True``, :8); this build has no network, so
weights come from a local file (``--vgg_weights`` / ``DSGAN_VGG16_WEIGHTS``) or, failing that,
a deterministic He-normal init (stated loudly; the perceptual term is then not the
reference's, see SURVEY.md §8c "parity unpinned").

relu5_3 is not used by the loss (DSGAN/models/pix2pix_model.py:182-186 uses features 0..3), so
its block is skipped unless ``with_relu5_3=True``.
"""
import math
import os

import torch
import torch.nn as nn

from dsgan_hip import functional as HF

_CFG = [("to_relu_1_2", [(0, 3, 64), (2, 64, 64)], False),
        ("to_relu_2_2", [(5, 64, 128), (7, 128, 128)], True),
        ("to_relu_3_3", [(10, 128, 256), (12, 256, 256), (14, 256, 256)], True),
        ("to_relu_4_3", [(17, 256, 512), (19, 512, 512), (21, 512, 512)], True),
        ("to_relu_5_3", [(24, 512, 512), (26, 512, 512), (28, 512, 512)], True)]


class Vgg16(nn.Module):
    def __init__(self, weights_path=None, seed=7000):
        super().__init__()
        for name, convs, _ in _CFG:
            seq = nn.Sequential()
            for idx, ci, co in convs:
                seq.add_module(str(idx), nn.Conv2d(ci, co, kernel_size=3, padding=1))
            setattr(self, name, seq)
        path = weights_path or os.environ.get("DSGAN_VGG16_WEIGHTS")
        if path:
            self.load_vgg_weights(path)
        else:
            self.synthetic_init(seed)
        for p in self.parameters():
            p.requires_grad = False

    @torch.no_grad()
    def synthetic_init(self, seed):
        print("[Vgg16] ImageNet weights unavailable offline: deterministic He-normal init "
              "(pass --vgg_weights / DSGAN_VGG16_WEIGHTS for the real perceptual loss)")
        for i, (k, p) in enumerate(self.named_parameters()):
            g = torch.Generator().manual_seed(seed + i)
            if k.endswith("bias"):
                p.copy_(0.01 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(math.sqrt(2.0 / (p.shape[1] * 9)) * torch.randn(p.shape, generator=g))

    def load_vgg_weights(self, path):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if any(k.startswith("features.") for k in sd):
            remap = {}
            for name, convs, _ in _CFG:
                for idx, _, _ in convs:
                    for t in ("weight", "bias"):
                        remap["%s.%d.%s" % (name, idx, t)] = sd["features.%d.%s" % (idx, t)]
            sd = remap
        self.load_state_dict(sd, strict=True)

    def forward(self, x, with_relu5_3=False):
        feats = []
        h = x
        for name, convs, pool in _CFG:
            if name == "to_relu_5_3" and not with_relu5_3:
                feats.append(None)
                break
            if pool:
                h = HF.max_pool2d(h, 2)
            seq = getattr(self, name)
            for idx, _, _ in convs:
                c = seq._modules[str(idx)]
                h = HF.conv2d(h, c.weight, c.bias, stride=1, pad=1, act="relu")
            feats.append(h)
        return tuple(feats)

    def loss_blocks(self):
        """[(pool, [(w, b), ...])] of the four blocks the perceptual loss reads (relu1_2..relu4_3)."""
        out = []
        for name, convs, pool in _CFG[:4]:
            seq = getattr(self, name)
            out.append((pool, [(seq._modules[str(i)].weight, seq._modules[str(i)].bias) for i, _, _ in convs]))
        return out

    @torch.no_grad()
    def loss_features(self, x):
        """relu1_2..relu4_3 of x without autograd (the real-image side of the perceptual loss):
        fp32 CB16 tensors from the channel-blocked bf16 pass (vggconv.hip) when the precision and
        image size allow it, NCHW fp32 otherwise -- perceptual_l1 follows the same choice."""
        if HF.vgg_cb16_ok(x):
            return HF.vgg_features_cb16(x, self.loss_blocks())[0]
        return HF.vgg_features_raw(x, self.loss_blocks())[0]

    def perceptual_l1(self, fake, real_feats, side=None):
        """L1(f1,r1) + L1(f2,r2) + L1(f3,r3) + L1(f0,r0) of f = self(fake), r = real_feats
        (DSGAN/models/pix2pix_model.py:180-186) as one fused autograd node; side (nullable stream):
        where its forward's kernels run (functional.perceptual_l1)."""
        return HF.perceptual_l1(fake, self.loss_blocks(), list(real_feats), side)

