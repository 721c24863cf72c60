"""Deterministic weight recipes for parity runs -- TEST INFRASTRUCTURE ONLY.

Golden fixtures ship a *recipe* instead of ~90 MB of weights.
For the i-th entry of a parameter list (reference ``state_dict`` order):

* ``"ref"``   -- the reference's own init statistics (``init_weights`` 'normal',
  DSGAN/models/networks.py:49-70: N(0, 0.02) conv/linear weights), except that
  biases get 0.01*N(0,1) (the reference zeros them; non-zero biases exercise the
  bias paths) and PReLU keeps its 0.25 default;
* ``"fanin"`` -- N(0, 1/fan_in) weights (a well-conditioned regime where every
  InstanceNorm input has variance >> eps, so fp32 gradients are meaningful),
  biases 0.1*N(0,1), PReLU 0.25;
* ``"vgg"``   -- N(0, 2/fan_in) weights, 0.01*N(0,1) biases (stand-in for the
  unavailable ImageNet VGG16 weights, DSGAN/models/vgg.py:8).

Each tensor is drawn from its own ``torch.Generator().manual_seed(seed0 + i)`` so
a value never depends on how many tensors precede it in a different process.
"""
from collections import OrderedDict
import math

import torch


def make_params(spec, recipe="ref", seed0=1000, dtype=torch.float32):
    out = OrderedDict()
    for i, (name, shape) in enumerate(spec):
        g = torch.Generator().manual_seed(seed0 + i)
        if name.endswith("relu1.weight"):
            t = torch.full(shape, 0.25)
        elif name.endswith(".bias"):
            s = {"ref": 0.01, "fanin": 0.1, "vgg": 0.01}[recipe]
            t = s * torch.randn(shape, generator=g)
        else:
            fan_in = int(math.prod(shape[1:])) if len(shape) > 1 else 1
            if recipe == "ref":
                std = 0.02
            elif recipe == "fanin":
                std = 1.0 / math.sqrt(fan_in)
            elif recipe == "vgg":
                std = math.sqrt(2.0 / fan_in)
            else:
                raise ValueError(recipe)
            t = std * torch.randn(shape, generator=g)
        out[name] = t.to(dtype)
    return out


def synth_pair(batch, size, seed=0):
    """Synthetic TIR/RGB pair, SURVEY.md §8d: u8 uniform, TIR gray replicated x3,
    normalised as (u8/255-0.5)/0.5 (DSGAN/data/aligned_dataset.py:53-63)."""
    g = torch.Generator().manual_seed(seed)
    tir = torch.randint(0, 256, (batch, 1, size, size), generator=g, dtype=torch.uint8)
    rgb = torch.randint(0, 256, (batch, 3, size, size), generator=g, dtype=torch.uint8)
    A = ((tir.float() / 255.0 - 0.5) / 0.5).repeat(1, 3, 1, 1)
    B = (rgb.float() / 255.0 - 0.5) / 0.5
    return A.contiguous(), B.contiguous()


def probe(numel, seed):
    """Seeded probe vector used for linear checksums of large gradient tensors."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn(numel, generator=g, dtype=torch.float64)
