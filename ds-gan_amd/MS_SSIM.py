"""SSIM / MS-SSIM on the HIP path (DSGAN/MS_SSIM.py:95-225 interface).

``ssim(X, Y, data_range, size_average=True)`` with the default 11-tap sigma-1.5 gaussian runs
the fused SSIM kernel (forward + analytic backward).  ``ms_ssim`` (DSGAN/MS_SSIM.py:153-225)
runs the MS-SSIM kernels: five scales of the SSIM / contrast-structure plane means with the
padded 2x2 average pool between them, combined on the device.  Both are differentiable like the
reference's autograd versions: when one operand requires grad the training kernels run
(``HF.SSIMFn`` / ``HF.MSSSIMFn``, analytic backward through the gaussian filters and the
pyramid) and the gradient flows to that operand.  SSIM is symmetric in (X, Y), so the operand
that requires grad is passed as the kernels' differentiated argument.  A gradient w.r.t. both
operands at once is not implemented and raises (never a silent zero gradient); without any
operand requiring grad, ``ms_ssim`` uses the evaluation kernel (per-image values for
``size_average=False``).
"""
import torch

from dsgan_hip import functional as HF


def _grad_order(X, Y, name):
    """(const, differentiated) operands, or None when no grad is needed."""
    need = torch.is_grad_enabled()
    gx, gy = need and X.requires_grad, need and Y.requires_grad
    if gx and gy:
        raise NotImplementedError("HIP %s differentiates w.r.t. one operand; both X and Y require grad" % name)
    if gy:
        return X, Y
    if gx:
        return Y, X     # SSIM(X, Y) == SSIM(Y, X): differentiate the X side
    return None


def ssim(X, Y, data_range=255, size_average=True, win_size=11, win_sigma=1.5, win=None,
         K=(0.01, 0.03), nonnegative_ssim=False):
    if X.shape != Y.shape:
        raise ValueError(f"Input images should have the same dimensions, but got {X.shape} and {Y.shape}.")
    if X.dim() != 4:
        raise ValueError("HIP ssim supports 4-d (N,C,H,W) tensors")
    if win is not None or win_size != 11 or win_sigma != 1.5 or tuple(K) != (0.01, 0.03):
        raise NotImplementedError("HIP ssim implements the default window (11, 1.5) and K=(0.01, 0.03)")
    if not size_average or nonnegative_ssim:
        raise NotImplementedError("HIP ssim implements size_average=True without relu")
    order = _grad_order(X, Y, "ssim")
    real, fake = order if order is not None else (X, Y)
    return HF.ssim_affine(real, fake, 1.0, 0.0, float(data_range))


def ms_ssim(X, Y, data_range=255, size_average=True, win_size=11, win_sigma=1.5, win=None, weights=None,
            K=(0.01, 0.03)):
    if X.shape != Y.shape:
        raise ValueError(f"Input images should have the same dimensions, but got {X.shape} and {Y.shape}.")
    if X.dim() != 4:
        raise ValueError("HIP ms_ssim supports 4-d (N,C,H,W) tensors")
    if win is not None or win_size != 11 or win_sigma != 1.5 or tuple(K) != (0.01, 0.03):
        raise NotImplementedError("HIP ms_ssim implements the default window (11, 1.5) and K=(0.01, 0.03)")
    w = HF.MS_SSIM_WEIGHTS if weights is None else tuple(float(v) for v in weights)
    smaller_side = min(X.shape[-2:])
    assert smaller_side > (win_size - 1) * (2 ** (len(w) - 1)), \
        "Image size should be larger than %d due to the 4 downsamplings in ms-ssim" % ((win_size - 1) * (2 ** 4))
    order = _grad_order(X, Y, "ms_ssim")
    if order is None:
        return HF.ms_ssim_affine(X, Y, 1.0, 0.0, float(data_range), w, size_average)
    if not size_average:
        raise NotImplementedError("HIP ms_ssim gradient implements size_average=True (the batch mean)")
    real, fake = order
    return HF.ms_ssim_loss_affine(real, fake, 1.0, 0.0, float(data_range), w)
