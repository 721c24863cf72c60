"""dsgan_hip -- MI355X-native kernels for the DS-GAN G+D train step.

The compute path is libdsgan_hip.so (HIP, gfx950), reached through the C-ABI in
include/dsgan_hip.h.  This package is the thin Python host layer: a ctypes binding
(``_lib``), autograd Functions composing the fused kernels (``functional``), flat parameter
buffers + fused Adam (``flat``) and the data-parallel gradient exchange (``dist``).
"""
from ._lib import load, LIB_PATH  # noqa: F401
from .functional import set_precision, get_precision  # noqa: F401


def require_gpu():
    """Fail loudly if the HIP path cannot run (no silent CPU fallback anywhere)."""
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("dsgan_hip: no ROCm GPU visible; the DS-GAN hot path runs only on MI355X")
    load()
