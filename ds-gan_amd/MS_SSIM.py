"""SSIM on the HIP path (DSGAN/MS_SSIM.py:95-150 interface).

``ssim(X, Y, data_range, size_average=True)`` with the default 11-tap sigma-1.5 gaussian runs
the fused SSIM kernel (forward + analytic backward w.r.t. Y).  ``ms_ssim`` (DSGAN/MS_SSIM.py:153-225,
the evaluation metric) runs the MS-SSIM kernels: five scales of the SSIM /
contrast-structure plane means with the padded 2x2 average pool between them, combined on the
device; it is not differentiable (the reference never back-propagates through it).
"""
from dsgan_hip import functional as HF


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
    if X.requires_grad:
        raise NotImplementedError("HIP ssim differentiates w.r.t. Y only (the generated image)")
    return HF.ssim_affine(X, Y, 1.0, 0.0, float(data_range))


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
    return HF.ms_ssim_affine(X, Y, 1.0, 0.0, float(data_range), w, size_average)
