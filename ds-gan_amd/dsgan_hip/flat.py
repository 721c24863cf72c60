"""Flat parameter / gradient buffers and the fused Adam that updates them.

All parameters of one network live in ONE contiguous fp32 device buffer (each ``Parameter`` is
a view into it), and all their gradients in a second one.  That gives:
  * one Adam launch per network per step (``dsgan_adam``),
  * one zeroing launch per network per step,
  * a flat gradient to all-reduce across ranks in a few large RCCL buckets
    (one process per GPU; see ``dsgan_hip.dist``).
State-dict keys and shapes are untouched, so reference checkpoints load unchanged.
"""
import torch

from ._lib import call, ptr, stream
from .functional import fill_, bump_weight_generation


class FlatParams:
    """``order`` (optional): the modules whose parameters come first in the buffer, in that order
    (the rest follow in ``module.parameters()`` order).  The generator passes its backward order
    so that the gradient buckets of dsgan_hip.dist.GradBuckets fill front to back."""

    def __init__(self, module, device, order=None):
        self.params = [p for p in module.parameters()]
        placed = []
        if order:
            seen = set()
            for m in order:
                for p in m.parameters():
                    if id(p) not in seen:
                        seen.add(id(p))
                        placed.append(p)
            placed += [p for p in self.params if id(p) not in seen]
        else:
            placed = list(self.params)
        assert len(placed) == len(self.params)
        # every tensor starts on a 256-byte boundary (vector loads in the kernels)
        offs, n = {}, 0
        self.layout = []
        for p in placed:
            offs[id(p)] = n
            self.layout.append((p, n, p.numel()))
            n += (p.numel() + 63) // 64 * 64
        offs = [offs[id(p)] for p in self.params]
        self.numel = n
        self.data = torch.empty(n, device=device, dtype=torch.float32)
        self.grad = torch.empty(n, device=device, dtype=torch.float32)
        fill_(self.data, 0.0)
        with torch.no_grad():
            for p, off in zip(self.params, offs):
                k = p.numel()
                self.data[off:off + k].copy_(p.detach().reshape(-1).to(device=device, dtype=torch.float32))
                p.data = self.data[off:off + k].view(p.shape)
                p.grad = self.grad[off:off + k].view(p.shape)
        self.zero_grad()

    def zero_grad(self):
        fill_(self.grad, 0.0)


class FlatAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False, weight_decay=0) over a FlatParams buffer in one kernel.

    Subclasses torch.optim.Optimizer so the reference's LambdaLR scheduler (get_scheduler,
    DSGAN/models/networks.py:33-46) drives ``param_groups[0]['lr']`` exactly as before.
    """

    def __init__(self, flat, lr=2e-4, betas=(0.9, 0.999), eps=1e-8, scaler=None):
        super().__init__(flat.params, dict(lr=lr, betas=betas, eps=eps))
        self.flat = flat
        self.scaler = scaler   # dsgan_hip.amp.LossScaler (--precision fp16): unscale / skip on device
        self.m = torch.zeros_like(flat.data)
        self.v = torch.zeros_like(flat.data)
        self.step_count = 0

    def zero_grad(self, set_to_none=False):
        self.flat.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        self.step_count += 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        if self.scaler is not None:
            # the scaler's check() has run on this gradient: g / scale, skipped on overflow, its
            # own step count for the bias corrections (step_count here counts calls)
            call("dsgan_adam_amp", ptr(self.flat.data), ptr(self.flat.grad), ptr(self.m), ptr(self.v),
                 self.flat.numel, float(g["lr"]), float(b1), float(b2), float(g["eps"]), ptr(self.scaler.state),
                 stream())
        else:
            call("dsgan_adam", ptr(self.flat.data), ptr(self.flat.grad), ptr(self.m), ptr(self.v),
                 self.flat.numel, float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                 self.step_count, stream())
        bump_weight_generation(self.flat.params)
        return None
