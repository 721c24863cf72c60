"""ctypes binding of libdsgan_hip.so (the C-ABI declared in include/dsgan_hip.h).

There is no fallback: if the library is missing or fails to load, every op raises.  The
signature table below is the single source of truth on the Python side and is checked
against include/dsgan_hip.h by tests/test_capi.py.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DSGAN_HIP_LIB", os.path.join(_HERE, "libdsgan_hip.so"))

P = ctypes.c_void_p
L = ctypes.c_long
I = ctypes.c_int
F = ctypes.c_float
D = ctypes.c_double
S = ctypes.c_void_p  # hipStream_t

SIGNATURES = {
    "dsgan_abi_version": [],
    "dsgan_set_half_type": [ctypes.c_int],
    "dsgan_amp_parts": [],
    "dsgan_amp_check": [P, L, P, P, F, F, I, S],
    "dsgan_adam_amp": [P, P, P, P, L, D, D, D, D, P, S],
    "dsgan_get_half_type": [],
    "dsgan_clear_launch_error": [],
    "dsgan_ktimer": [I],
    "dsgan_ktimer_read": [P, I],
    "dsgan_last_error_string": [],
    # scratch contract: plan-only mode and the scratch the last planned launch needs (CPU planner tests)
    "dsgan_set_plan_only": [I],
    "dsgan_last_ws_need": [],
    # igemm.hip
    "dsgan_conv_fwd": [P, L, P, P, P, L, P, L] + [I] * 12 + [F, I, I, I, S],
    "dsgan_conv_dgrad": [P, L, P, P, P, L, P, L, P, L, I, I, I, I, I, I, I, I, I, I, I, I, I, F, I, I, S],
    "dsgan_conv_wgrad": [P, L, P, L, P] + [I] * 13 + [P, L, S],
    "dsgan_conv_wgrad_workspace": [I] * 8,
    # pwgemm.hip
    "dsgan_pw_supported": [I, I, I, I, L, L, P, P],
    "dsgan_pw_gemm": [I, P, L, P, L, P, L, P, P, L, P, L, I, I, I, I, I, I, I, I, I, F, P, L, S],
    "dsgan_pw_wgrad_workspace": [I, I, I, I],
    "dsgan_pw_wgrad_mixed": [P, L, I, P, L, I, P, P, I, I, I, I, P, L, S],
    "dsgan_pw_fwd_io": [P, I, P, L, I, P, L, I, P, L, I, P, I, I, I, I, I, I, F, S],
    "dsgan_pw_dgrad_io": [P, I, P, L, I, P, L, I, P, L, I, I, I, I, I, S],
    "dsgan_pw_fwd_io_ws": [P, I, P, L, I, P, L, I, P, L, I, P, I, I, I, I, I, I, F, P, L, S],
    "dsgan_pw_dgrad_io_ws": [P, I, P, L, I, P, L, I, P, L, I, I, I, I, I, P, L, S],
    "dsgan_pw_fd_workspace": [I, I, I, I, I],
    "dsgan_wtrans_multi": [P, P, P, I, S],
    "dsgan_pw_tune": [I, I],
    # pwf32.hip
    "dsgan_pw_f32_supported": [I, I, I, I, L, L, P, P],
    "dsgan_pw_f32_wgrad_workspace": [I, I, I, I],
    "dsgan_pw_gemm_f32": [I, P, L, P, L, P, L, P, P, L, I, I, I, I, I, I, I, I, F, P, L, S],
    # mlp.hip
    "dsgan_mlp_supported": [I, I, I],
    "dsgan_mlp_fwd": [P, L, I, P, P, P, P, P, L, I, I, I, I, I, S],
    "dsgan_mlp_bwd": [P, L, I, P, L, P, P, P, P, L, P, P, P, I, I, I, I, S],
    "dsgan_mlp_wgrad_workspace": [I, I, I, I],
    "dsgan_mlp_wgrad": [P, L, I, P, L, P, P, P, P, P, P, P, L, I, I, I, I, S],
    "dsgan_mlp_tune": [I, I],
    "dsgan_colsum": [P, I, I, P, S],
    # split_reduce.hip: deferred split reductions (one batched flush per backward pass)
    "dsgan_split_defer": [I],
    "dsgan_split_pending": [],
    "dsgan_split_flush": [S],
    "dsgan_f32_to_bf16": [P, P, L, S],
    # pconv.hip
    "dsgan_pconv_supported": [I, I, I, I],
    "dsgan_conv_wtrans_bf16": [P, P, I, I, I, I, I, S],
    "dsgan_pconv": [P, L, P, P, P, L, P, L] + [I] * 13 + [F, I, S],
    "dsgan_pconv_workspace": [I] * 5,
    "dsgan_pconv_ws": [P, L, P, P, P, L, P, L] + [I] * 13 + [F, I, P, L, S],
    # pwsmall.hip
    "dsgan_pw_small_supported": [I, I, I, L, L],
    "dsgan_pw_small": [P, L, P, I, I, P, P, L, P, L] + [I] * 8 + [F, S],
    "dsgan_pw_small2": [P, L, P, I, I, P, L, P, I, P, P, L, P, L] + [I] * 8 + [F, S],
    # pconvt.hip
    "dsgan_pconvt_supported": [I, I, I, I],
    "dsgan_pconvt": [P, L, P, P, P, L, P, L] + [I] * 11 + [F, I, S],
    # wconv.hip
    "dsgan_wconv_supported": [I, I, I, I],
    "dsgan_wconv_workspace": [I, I, I, I, I, I, I],
    "dsgan_wconv": [P, L, P, L, P, P, L] + [I] * 11 + [S],
    "dsgan_wconv_db": [P, L, P, L, P, P, P, L] + [I] * 11 + [S],
    "dsgan_wconv_xh": [P, L, P, L, P, P, L] + [I] * 11 + [S],
    # tconv.hip
    "dsgan_conv_wtrans": [P, P, I, I, I, I, I, I, I, I, I, S],
    "dsgan_tconv": [P, L, P, P, P, L, P, L] + [I] * 9 + [P, P] + [I] * 7 + [F, S],
    "dsgan_tconv_workspace": [I] * 6,
    "dsgan_tconv_ws": [P, L, P, P, P, L, P, L] + [I] * 9 + [P, P] + [I] * 7 + [F, I, P, L, S],
    "dsgan_tconv_ws_xh": [P, L, P, P, P, L, P, L] + [I] * 9 + [P, P] + [I] * 7 + [F, P, L, S],
    # skinny.hip
    "dsgan_conv_small_out": [P, L, P, L, L, L, L, P, P, L] + [I] * 13 + [S],
    "dsgan_conv_small_in": [P, L, P, L, L, L, L, P, P, L] + [I] * 13 + [F, I, S],
    "dsgan_conv_wgrad_small_workspace": [I] * 7,
    "dsgan_conv_wgrad_small": [P, L, P, L, P] + [I] * 11 + [P, L, S],
    # thin3.hip
    "dsgan_thin3_supported": [I, I, I, L, L],
    "dsgan_pgstem_supported": [I] * 4,
    "dsgan_pgstem_fwd": [P, L, P, P, P, L] + [I] * 5 + [F, S],
    "dsgan_pgstem_wgrad_workspace": [I] * 5,
    "dsgan_pgstem_wgrad": [P, L, P, L, P, L, P, P] + [I] * 5 + [F, P, L, S],
    "dsgan_pgstem_dgrad": [P, L, P, L, P, P, L] + [I] * 5 + [F, I, S],
    "dsgan_pglast_supported": [I] * 3,
    "dsgan_pglast_workspace": [I] * 4,
    "dsgan_pglast_fwd": [P, L, P, P, P, L] + [I] * 5 + [P, L, S],
    "dsgan_pglast_wgrad": [P, L, P, L, P, P] + [I] * 4 + [P, L, S],
    "dsgan_pglast_dgrad": [P, L, P, P, L] + [I] * 5 + [S],
    "dsgan_thin3_fwd": [P, L, P, P, P, L] + [I] * 6 + [S],
    "dsgan_thin3_wgrad_workspace": [I] * 5,
    "dsgan_thin3_wgrad": [P, L, P, L, P, P, L] + [I] * 5 + [S],
    "dsgan_thin3_dgrad": [P, L, P, P, L] + [I] * 6 + [S],
    # dwconv.hip
    "dsgan_dwconv_fwd": [P, L, P, P, P, L, I, I, I, I, I, I, I, S],
    "dsgan_dwconv_wgrad_workspace": [I, I, I, I, I, I],
    "dsgan_dwconv_wgrad": [P, L, P, L, P, P, I, I, I, I, I, P, L, S],
    "dsgan_dwconv_multi_supported": [I, I, P, L, P, L],
    "dsgan_dwconv_multi_fwd": [P, L, P, P, P, P, P, P, P, P, P, L, I, I, I, I, I, I, S],
    "dsgan_dwconv_multi_wgrad_workspace": [I, I, I, I],
    "dsgan_dwconv_multi_wgrad": [P, L, P, L, P, P, P, P, P, P, P, P, I, I, I, I, P, L, S],
    # norm_pointwise.hip
    "dsgan_instnorm_fwd": [P, L, P, P, L, P, L, P, P, I, I, I, I, F, F, S],
    "dsgan_instnorm_fwd_bf16": [P, L, P, L, P, P, I, I, I, F, S],
    "dsgan_instnorm_bwd": [P, L, P, L, P, P, L, P, P, P, L, P, L, P, I, I, I, I, F, F, S],
    "dsgan_instnorm_bwd_h": [P, L, P, L, P, L, P, P, P, L, P, P, L, I, I, I, I, F, F, S],
    "dsgan_instnorm_workspace": [I, I, I],
    "dsgan_instnorm_fwd_ws": [P, L, P, P, L, P, L, P, P, I, I, I, I, F, F, P, L, S],
    "dsgan_instnorm_bwd_ws": [P, L, P, L, P, P, L, P, P, P, L, P, L, P, I, I, I, I, F, F, P, L, S],
    "dsgan_maxpool_fwd": [P, L, P, L, P, I, I, I, I, I, S],
    "dsgan_maxpool_bwd": [P, L, P, P, L, I, I, I, I, I, I, S],
    "dsgan_maxpool_pyr_supported": [I, I, I],
    "dsgan_maxpool_pyr_fwd": [P, L, I] + [P] * 8 + [I, I, I, I, S],
    "dsgan_maxpool_pyr_bwd": [P, L, P] * 4 + [P, L] + [I] * 6 + [S],
    "dsgan_plane_stats": [P, L, P, P, P, I, I, I, S],
    "dsgan_plane_stats_bwd": [P, P, P, P, L, I, I, I, S],
    "dsgan_ca_fwd": [P, P, P, P, P, P, P, I, I, I, S],
    "dsgan_ca_bwd": [P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, P, L, S],
    "dsgan_add_n": [P, P, I, P, L, I, L, S],
    "dsgan_copy_strided": [P, L, P, L, I, L, S],
    "dsgan_copy_multi": [P, P, I, L, S],
    "dsgan_fill": [P, F, L, S],
    "dsgan_scale": [P, F, L, S],
    "dsgan_act_bwd": [P, P, P, L, I, F, I, S],
    "dsgan_channel_sum": [P, L, P, I, I, I, P, L, S],
    # losses.hip
    "dsgan_loss_parts": [],
    "dsgan_loss_combine": [P, P, P, P, I, F, P, S],
    "dsgan_loss_combine_bwd": [P, P, P, I, F, P, S],
    "dsgan_ssim_parts": [I, I, I],
    "dsgan_bce_logits_fwd": [P, L, F, P, P, S],
    "dsgan_bce_logits_bwd": [P, L, F, P, P, I, S],
    "dsgan_l1_fwd": [P, P, L, P, P, S],
    "dsgan_l1_bwd": [P, P, L, P, P, I, S],
    "dsgan_vgg_tap_bwd": [P, P, P, P, P, L, I, I, P, S],
    "dsgan_tv_fwd": [P, L, I, I, F, P, P, S],
    "dsgan_tv_bwd": [P, L, I, I, F, P, P, I, S],
    "dsgan_ssim_fwd": [P, P, F, F, I, I, I, P, F, F, P, P, P, S],
    "dsgan_ms_ssim_workspace": [I, I, I, I],
    "dsgan_u8_to_image": [P, P, P, I, I, I, I, S],
    "dsgan_img_metrics": [P, P, I, I, I, P, P, S],
    "dsgan_ms_ssim": [P, P, F, F, I, I, I, I, P, F, F, P, I, P, L, P, P, S],
    "dsgan_ms_ssim_train_workspace": [I, I, I, I, I],
    "dsgan_ms_ssim_fwd_train": [P, P, F, F, I, I, I, I, P, F, F, P, I, P, L, P, P, S],
    "dsgan_ms_ssim_bwd": [P, P, F, F, I, I, I, I, P, F, F, P, I, P, L, P, P, P, I, S],
    "dsgan_ssim_bwd": [P, P, F, F, I, I, I, P, P, P, F, P, I, S],
    # vggconv.hip
    "dsgan_vconv_supported": [I, I, I, I],
    "dsgan_vconv_tune": [I, I],
    "dsgan_vconv_wtrans_size": [I, I],
    "dsgan_vconv_wtrans": [P, P, I, I, I, S],
    "dsgan_vconv3x3": [P, P, P, P, P, I, I, I, I, I, I, I, S],
    "dsgan_vgg_conv1_fwd": [P, L, P, P, P, I, I, I, S],
    "dsgan_vgg_conv1_dgrad": [P, P, P, L, I, I, I, S],
    "dsgan_cb16_maxpool": [P, P, P, I, I, I, I, S],
    "dsgan_cb16_maxpool_l1": [P, P, P, P, P, P, P, L, I, I, I, I, S],
    "dsgan_cb16_tap_bwd_codes": [P, P, P, P, I, I, I, I, P, S],
    "dsgan_cb16_maxpool_l1_parts": [I, I, I, I],
    "dsgan_cb16_tap_bwd": [P, P, P, P, P, I, I, I, I, P, S],
    # adam.hip
    "dsgan_adam": [P, P, P, P, L, D, D, D, D, I, S],
}

_lib = None


def load():
    """Load the library (idempotent).  Raises RuntimeError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            "libdsgan_hip.so not found at %s -- build it with `python ds-gan_amd/build_lib.py` "
            "(there is no CPU/PyTorch fallback for the DS-GAN hot path)" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = (ctypes.c_char_p if name == "dsgan_last_error_string"
                      else ctypes.c_long if name.endswith(("_workspace", "_parts", "_size", "_need")) else ctypes.c_int)
    _lib = lib
    return lib


# Set by functional.deferred_splits(): called after every entry point with whether that call queued
# a deferred split reduction (dsgan_split_pending rose), so that only the scratch of a call that
# queued one is kept alive until the flush.
DEFER_HOOK = [None]


def call(name, *args):
    lib = load()
    hook = DEFER_HOOK[0]
    n0 = lib.dsgan_split_pending() if hook is not None else 0
    rc = getattr(lib, name)(*args)
    if hook is not None:
        hook(lib.dsgan_split_pending() > n0)
    if rc != 0:
        msg = lib.dsgan_last_error_string()
        raise RuntimeError("%s failed (rc=%d): %s" % (name, rc, msg.decode() if msg else ""))


def ptr(t):
    """Device pointer of a tensor (None -> NULL).  Refuses CPU tensors: the product path is GPU-only."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("dsgan_hip: expected a device tensor, got %s on %s" % (tuple(t.shape), t.device))
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream
