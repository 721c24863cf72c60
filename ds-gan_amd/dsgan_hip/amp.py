"""Dynamic loss scaling for ``--precision fp16`` (BASELINE configs[4]), device-resident.

The reference trains in fp32 (DSGAN/models/pix2pix_model.py:201-217).  In the fp16 mode every
16-bit MFMA operand of the backward -- upstream gradients, the MLP's dz, the VGG data-grads --
is an IEEE half, whose normal range ends at 6.1e-5: a batch-mean loss over 8 x 3 x 512 x 512
pixels has per-pixel gradients of ~1.6e-7, deep in the subnormals.  As with
torch.cuda.amp.GradScaler the loss is multiplied by a power-of-two scale before backward (exact
in fp32), so the backward runs in the normal fp16 range, and the optimizer sees the gradient
divided by it again.  Unlike GradScaler nothing here syncs with the host:

  * ``scale(loss)`` multiplies by the device scalar ``state[0]``;
  * ``check(flat_grad)`` (after the backward and the DDP all-reduce) scans the flat gradient
    for inf / nan and updates the state in one tiny kernel (dsgan_amp_check): an overflowed step
    is marked skipped and the scale halves; after ``growth_interval`` clean steps it doubles;
  * ``FlatAdam.step`` then runs dsgan_adam_amp, which divides by the step's scale and does
    nothing on a skipped step (its bias-correction step count, ``state[4]``, is not advanced --
    GradScaler skips optimizer.step()).
One scaler per network (D and G have their own backward and optimizer).  Defaults are
GradScaler's (init 2^16, growth 2, backoff 0.5, interval 2000).

``LossScaler.guard(device)`` is the unit-scale form (scale 1, never grown or backed off): the bf16
mode's non-finite guard (``--nonfinite_guard``).  ``scale`` is then the identity, the check and the
skip are the same kernels, and Adam multiplies the gradient by exactly 1.0.
"""
import torch

from . import _lib
from ._lib import call, ptr, stream


class LossScaler:
    def __init__(self, device, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000):
        # {scale, skip, clean steps, 1/scale of the last checked step, applied optimizer steps}
        self.state = torch.tensor([init_scale, 0.0, 0.0, 1.0 / init_scale, 0.0], device=device, dtype=torch.float32)
        self.part = torch.empty(int(_lib.load().dsgan_amp_parts()), device=device, dtype=torch.int32)
        self.growth, self.backoff, self.interval = float(growth_factor), float(backoff_factor), int(growth_interval)

    @classmethod
    def guard(cls, device):
        s = cls(device, init_scale=1.0, growth_factor=1.0, backoff_factor=1.0, growth_interval=1 << 30)
        s.unit = True
        return s

    unit = False

    def scale(self, loss):
        """loss * scale (a power of two: exact); the scale is a device scalar, no host sync."""
        return loss if self.unit else loss * self.state[0]

    def skipped_steps(self, calls):
        """optimizer steps skipped so far out of `calls` (synchronises)"""
        return calls - self.applied_steps()

    def check(self, flat_grad):
        call("dsgan_amp_check", ptr(flat_grad), flat_grad.numel(), ptr(self.part), ptr(self.state), self.backoff,
             self.growth, self.interval, stream())

    # host-side views for logs / tests (these synchronise)
    def get_scale(self):
        return float(self.state[0].item())

    def skipped_last(self):
        return bool(self.state[1].item() != 0.0)

    def applied_steps(self):
        return int(self.state[4].item())
