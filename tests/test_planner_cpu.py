"""CPU planner tests of the scratch contract (include/dsgan_hip.h "Scratch contract").

Every scratch-taking entry point plans the launch it is about to issue and refuses a buffer smaller
than that plan writes.  In plan-only mode (dsgan_set_plan_only) the real launchers of
libdsgan_hip.so run their validation and planning on the host and return before any HIP call, so
these tests need no GPU.  For every pointwise planner knob setting (dsgan_pw_tune) and a sweep of
shapes covering the step's layers, the size the launcher needs is <= the size its *_workspace query
returns, and one element less is refused with an error code.

Round-3 regression: tools/pw_bench.py sized its split-K scratch with dsgan_pw_fd_workspace under
the default knobs and then launched with knob 2 = 512 (split launches of up to 512 tiles instead of
256): launches with 256-511 tiles split into a one-float buffer and the GPU faulted
(hipErrorIllegalAddress).  test_knob_change_after_query_is_refused replays that sequence: the
launch now returns -1.
"""
import ctypes
import itertools
import os

import numpy as np
import pytest

P16 = 16


@pytest.fixture(scope="module")
def lib():
    from dsgan_hip import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libdsgan_hip.so not built (run __graft_entry__.build())")
    lib = _lib.load()
    assert lib.dsgan_abi_version() == 3
    old = lib.dsgan_set_plan_only(1)
    assert old == 0
    yield lib
    lib.dsgan_set_plan_only(0)
    for k, v in DEFAULT_KNOBS.items():
        lib.dsgan_pw_tune(k, v)


# a host buffer standing in for every device operand: plan-only launchers check alignment and
# range but never dereference it
_BUF = np.zeros(1 << 16, dtype=np.uint8)
_BASE = (_BUF.ctypes.data + 255) // 256 * 256
A = _BASE          # 256-byte aligned "device" pointer
WS = _BASE + 4096  # scratch pointer (distinct, aligned)

DEFAULT_KNOBS = {0: 1, 1: 512, 2: 256, 3: 4, 4: 0, 5: 0, 6: 0, 7: 0, 8: 1}
KNOB_VALUES = {0: (0, 1), 1: (128, 512, 2048), 2: (64, 256, 512, 4096), 3: (1, 2, 4, 8), 4: (0, 1), 5: (0, 1),
               6: (0, 1, 2, 3), 7: (0, 1, 2, 3), 8: (0, 1)}


def knob_settings():
    """Every single-knob deviation from the defaults plus a few combined ones."""
    out = [dict(DEFAULT_KNOBS)]
    for k, vals in KNOB_VALUES.items():
        for v in vals:
            if v != DEFAULT_KNOBS[k]:
                d = dict(DEFAULT_KNOBS)
                d[k] = v
                out.append(d)
    out.append({**DEFAULT_KNOBS, 2: 4096, 3: 1, 4: 1, 5: 1})
    out.append({**DEFAULT_KNOBS, 1: 2048, 2: 4096, 6: 2, 7: 2})
    out.append({**DEFAULT_KNOBS, 2: 512, 4: 1, 6: 3, 7: 3, 8: 0})
    return out


def set_knobs(lib, knobs):
    for k, v in knobs.items():
        lib.dsgan_pw_tune(k, v)


def check(lib, fn, need_ws, args_before, args_after, name, optional=False):
    """fn(*args_before, ws, ws_elems, *args_after): passes with the queried size, and a buffer one
    element short of the launcher's own need is refused.  optional: NULL scratch is valid and
    means "never split" (the pointwise FWD / DGRAD, pconv and tconv split-K forms)."""
    rc = fn(*args_before, WS if need_ws > 0 else None, need_ws, *args_after)
    msg = lib.dsgan_last_error_string().decode()
    assert rc == 0, (name, msg)
    need = lib.dsgan_last_ws_need()
    assert 0 <= need <= need_ws, (name, need, need_ws)
    if need > 0:
        rc = fn(*args_before, WS, need - 1, *args_after)
        assert rc == -1 and "scratch of" in lib.dsgan_last_error_string().decode(), name
        rc = fn(*args_before, None, 0, *args_after)
        if optional:
            assert rc == 0 and lib.dsgan_last_ws_need() == 0, name
        else:
            assert rc == -1, name
    return need


# (M, K, HW) of the step's pointwise layers (MixConvNeXtML Blocks, shortcuts, downSkip, MLKA 1x1)
# plus off-grid shapes; nb = per-GPU batch
PW_SHAPES = [(m, k, hw) for m, k in [(256, 64), (64, 256), (512, 128), (128, 512), (1024, 256), (256, 1024),
                                     (2048, 512), (512, 2048), (4096, 1024), (1024, 4096), (64, 1024), (128, 1024),
                                     (96, 160), (48, 32)]
             for hw in (256, 1024, 4096, 16384, 65536)]
NBS = (1, 2, 8, 16, 32)


def _pw_fd_calls(lib, M, K, HW, nb):
    """(name, mode, callable(ws, ws_elems)) for every FWD / DGRAD form the step issues."""
    f = lib
    yield "pw_gemm fwd f32", 0, lambda ws, n: f.dsgan_pw_gemm(0, A, 0, A, K * HW, A, M * HW, None, None, 0, None, 0, M,
                                                              nb * HW, K, HW, nb, 0, 0, 0, 0, 0.2, ws, n, None)
    yield "pw_gemm dgrad f32 gact", 1, lambda ws, n: f.dsgan_pw_gemm(1, A, 0, A, K * HW, A, M * HW, None, None, 0, A,
                                                                    M * HW, M, nb * HW, K, HW, nb, 0, 1, 0, 0, 0.2, ws,
                                                                    n, None)
    if K % 8 == 0:
        yield "fwd_io gelu pair", 0, lambda ws, n: f.dsgan_pw_fwd_io_ws(A, 1, A, K * HW, 1, A, M * HW, 1, A, M * HW, 1, A,
                                                                       M, K, HW, nb, 1, 0, 0.2, ws, n, None)
        yield "fwd_io acc", 0, lambda ws, n: f.dsgan_pw_fwd_io_ws(A, 1, A, K * HW, 1, A, M * HW, 0, None, 0, 0, A, M, K,
                                                                 HW, nb, 0, 1, 0.2, ws, n, None)
    if M % 8 == 0:
        yield "dgrad_io gp", 1, lambda ws, n: f.dsgan_pw_dgrad_io_ws(A, 1, A, K * HW, 0, A, M * HW, 1, A, M * HW, M, K,
                                                                    HW, nb, 0, ws, n, None)
        yield "dgrad_io plain", 1, lambda ws, n: f.dsgan_pw_dgrad_io_ws(A, 1, A, K * HW, 1, A, M * HW, 0, None, 0, M, K,
                                                                       HW, nb, 0, ws, n, None)


def test_pw_fd_need_within_query_for_every_knob(lib):
    n_checked = n_split = 0
    for knobs in knob_settings():
        set_knobs(lib, knobs)
        for (M, K, HW), nb in itertools.product(PW_SHAPES, NBS):
            if HW % 128:
                continue
            for name, mode, call in _pw_fd_calls(lib, M, K, HW, nb):
                q = lib.dsgan_pw_fd_workspace(mode, M, K, HW, nb)
                need = check(lib, lambda ws, n: call(ws, n), q, (), (), (name, M, K, HW, nb, knobs), optional=True)
                n_checked += 1
                n_split += need > 0
    set_knobs(lib, DEFAULT_KNOBS)
    assert n_checked > 5000 and n_split > 100, (n_checked, n_split)


def test_pw_wgrad_need_within_query_for_every_knob(lib):
    n_split = 0
    for knobs in knob_settings():
        set_knobs(lib, knobs)
        for (M, N, HW), nb in itertools.product(PW_SHAPES, NBS):
            if nb * max(M, N) * HW * 4 >= 0xFFFFFFF0:   # beyond one buffer resource: refused up front
                continue
            q = lib.dsgan_pw_wgrad_workspace(M, N, HW, nb)
            for abf, bbf in ((0, 0), (0, 1), (1, 1)):
                need = check(lib, lambda ws, n: lib.dsgan_pw_wgrad_mixed(A, M * HW, abf, A, N * HW, bbf, A, A, M, N, HW,
                                                                         nb, ws, n, None),
                             q, (), (), ("wgrad_mixed", M, N, HW, nb, abf, bbf, knobs))
                n_split += need > 0
            check(lib, lambda ws, n: lib.dsgan_pw_gemm(2, A, M * HW, A, N * HW, A, 0, A, None, 0, None, 0, M, N,
                                                       nb * HW, HW, nb, 0, 0, 0, 0, 0.2, ws, n, None),
                  q, (), (), ("pw_gemm wgrad", M, N, HW, nb, knobs))
    set_knobs(lib, DEFAULT_KNOBS)
    assert n_split > 100


def test_knob_change_after_query_is_refused(lib):
    """The round-3 fault: scratch sized under the default knobs, launch under knob 2 = 512."""
    set_knobs(lib, DEFAULT_KNOBS)
    found = 0
    for (M, K, HW), nb in itertools.product(PW_SHAPES, NBS):
        q0 = lib.dsgan_pw_fd_workspace(1, M, K, HW, nb)
        lib.dsgan_pw_tune(2, 512)
        try:
            q1 = lib.dsgan_pw_fd_workspace(1, M, K, HW, nb)
            if q1 > q0:
                found += 1
                buf_elems = max(q0, 1)   # what pw_bench allocated: torch.empty(max(n, 1))
                rc = lib.dsgan_pw_gemm(1, A, 0, A, K * HW, A, M * HW, None, None, 0, None, 0, M, nb * HW, K, HW, nb,
                                       0, 0, 0, 0, 0.2, WS, buf_elems, None)
                assert rc == -1 and "scratch of" in lib.dsgan_last_error_string().decode()
                assert lib.dsgan_last_ws_need() == q1 > buf_elems
        finally:
            lib.dsgan_pw_tune(2, DEFAULT_KNOBS[2])
    assert found > 0


def test_conv_family_needs_within_queries(lib):
    """igemm / wconv / pconv / tconv / skinny / thin3 / dwconv / MLP / CA / channel-sum / MS-SSIM scratch."""
    for half in (0, 1):
        assert lib.dsgan_set_half_type(half) == 0
        for prec in (0, 1):
            for (N, Ci, Co, K, H, s) in [(16, 64, 128, 4, 128, 2), (16, 128, 256, 4, 64, 2), (16, 256, 512, 4, 32, 1),
                                         (2, 512, 1, 4, 31, 1), (16, 3, 64, 3, 256, 1), (4, 64, 64, 3, 16, 1)]:
                Ho = (H + 2 - K) // s + 1
                q = lib.dsgan_conv_wgrad_workspace(N, Ci, Co, K, K, Ho, Ho, prec)
                check(lib, lambda ws, n: lib.dsgan_conv_wgrad(A, Co * Ho * Ho, A, Ci * H * H, A, N, Ci, H, H, Co, K, K,
                                                              s, 1, Ho, Ho, 0, prec, ws, n, None),
                      q, (), (), ("conv_wgrad", N, Ci, Co, K, H, s, prec))
        # wconv: PatchGAN 4x4 s2/s1 and the ConvTranspose 3x3/s2 weight-grads, with / without the bias fold
        for (N, C, M, K, H, s) in [(16, 64, 128, 4, 128, 2), (16, 128, 256, 4, 64, 2), (16, 256, 512, 4, 32, 1),
                                   (16, 512, 256, 3, 32, 2), (16, 64, 32, 3, 256, 2), (3, 32, 96, 3, 16, 2),
                                   (1, 128, 256, 3, 20, 2)]:
            Ho = (H + 2 - K) // s + 1
            q = lib.dsgan_wconv_workspace(N, C, M, Ho, Ho, K, K)
            check(lib, lambda ws, n: lib.dsgan_wconv(A, M * Ho * Ho, A, C * H * H, A, ws, n, N, C, M, H, H, Ho, Ho, K,
                                                     K, s, 1, None), q, (), (), ("wconv", N, C, M, K, H, s))
            check(lib, lambda ws, n: lib.dsgan_wconv_db(A, M * Ho * Ho, A, C * H * H, A, A, ws, n, N, C, M, H, H, Ho,
                                                        Ho, K, K, s, 1, None), q, (), (), ("wconv_db", N, C, M, K, H, s))
            if K == 3 and s == 2:
                check(lib, lambda ws, n: lib.dsgan_wconv_xh(A, M * Ho * Ho, A, C * H * H, A, ws, n, N, C, M, H, H, Ho,
                                                            Ho, K, K, s, 1, None), q, (), (), ("wconv_xh", N, C, M, H))
        # pconv (split-K stride-1 PatchGAN layers, stride-2 forwards)
        for (N, Kc, M, KH, H, s) in [(16, 256, 512, 4, 32, 1), (16, 512, 256, 4, 33, 1), (16, 64, 128, 4, 128, 2),
                                     (16, 128, 256, 4, 64, 2), (2, 512, 256, 4, 33, 1), (64, 256, 512, 4, 32, 2),
                                     (64, 256, 512, 4, 32, 1), (4, 64, 64, 3, 32, 1)]:
            pad = 1
            Ho = (H + 2 * pad - KH) // s + 1
            q = lib.dsgan_pconv_workspace(N, Kc, M, Ho, Ho)
            check(lib, lambda ws, n: lib.dsgan_pconv_ws(A, Kc * H * H, A, None, A, M * Ho * Ho, None, 0, N, Kc, M, H, H,
                                                        Ho, Ho, KH, KH, s, pad, 0, 0, 0.2, 0, ws, n, None),
                  q, (), (), ("pconv", N, Kc, M, KH, H, s), optional=True)
        # tconv: the ConvTranspose data-grads at 16^2 / 32^2 and a filled launch
        taps = (ctypes.c_int * 9)(*([0] * 9))
        for (N, Kc, M, Ho) in [(16, 512, 1024, 16), (16, 256, 512, 32), (16, 64, 128, 128), (2, 1024, 512, 8)]:
            q = lib.dsgan_tconv_workspace(N, Kc, M, Ho, Ho, 9)
            check(lib, lambda ws, n: lib.dsgan_tconv_ws(A, Kc * Ho * Ho * 4, A, None, A, M * Ho * Ho, None, 0, N, Kc, M,
                                                        2 * Ho, 2 * Ho, Ho, Ho, 2, 9, ctypes.addressof(taps),
                                                        ctypes.addressof(taps), Ho, Ho, 1, 0, 0, 0, 0, 0.2, 1, ws, n,
                                                        None), q, (), (), ("tconv", N, Kc, M, Ho), optional=True)
            check(lib, lambda ws, n: lib.dsgan_tconv_ws_xh(A, Kc * Ho * Ho * 4, A, None, A, M * Ho * Ho, None, 0, N, Kc,
                                                           M, 2 * Ho, 2 * Ho, Ho, Ho, 2, 9, ctypes.addressof(taps),
                                                           ctypes.addressof(taps), Ho, Ho, 1, 0, 0, 0, 0, 0.2, ws, n,
                                                           None), q, (), (), ("tconv_xh", N, Kc, M, Ho), optional=True)
    lib.dsgan_set_half_type(0)
    # skinny / thin3 / pwf32 / MLP / depthwise / CA / channel sum / MS-SSIM
    for (N, Ci, Co, K, H) in [(16, 64, 3, 3, 256), (16, 512, 1, 4, 31), (16, 6, 64, 4, 256), (16, 3, 12, 1, 256)]:
        q = lib.dsgan_conv_wgrad_small_workspace(N, Ci, Co, K, K, H, H)
        check(lib, lambda ws, n: lib.dsgan_conv_wgrad_small(A, Co * H * H, A, Ci * H * H, A, N, Ci, H, H, Co, K, K, 1,
                                                            (K - 1) // 2, H, H, ws, n, None), q, (), (),
              ("wgrad_small", N, Ci, Co, K, H))
    for (N, K, M) in [(16, 64, 3), (2, 64, 3), (1, 33, 1)]:
        q = lib.dsgan_thin3_wgrad_workspace(N, K, M, 256, 256)
        check(lib, lambda ws, n: lib.dsgan_thin3_wgrad(A, M * 65536, A, K * 65536, A, ws, n, N, K, M, 256, 256, None),
              q, (), (), ("thin3", N, K, M))
    for (M, Nn, HW, nb) in [(256, 256, 256, 16), (128, 128, 1024, 16), (64, 64, 65536, 2), (512, 256, 4096, 16)]:
        q = lib.dsgan_pw_f32_wgrad_workspace(M, Nn, HW, nb)
        check(lib, lambda ws, n: lib.dsgan_pw_gemm_f32(2, A, M * HW, A, Nn * HW, A, 0, A, None, 0, M, Nn, nb * HW, HW,
                                                       nb, 0, 0, 0, 0.2, ws, n, None), q, (), (), ("pwf32", M, Nn, HW))
    for (C, P, HW, nb) in [(64, 128, 65536, 16), (128, 64, 16384, 16), (128, 256, 4096, 16), (256, 128, 1024, 16)]:
        if not lib.dsgan_mlp_supported(C, P, HW):
            continue
        q = lib.dsgan_mlp_wgrad_workspace(C, P, HW, nb)
        check(lib, lambda ws, n: lib.dsgan_mlp_wgrad(A, C * HW, 1, A, P * HW, A, A, A, A, A, A, ws, n, nb, C, P, HW,
                                                     None), q, (), (), ("mlp_wgrad", C, P, HW))
    for (N, C, H, K) in [(16, 64, 256, 7), (16, 256, 32, 7), (2, 48, 20, 5), (16, 1024, 16, 7)]:
        q = lib.dsgan_dwconv_wgrad_workspace(N, C, H, H, K, 1)
        check(lib, lambda ws, n: lib.dsgan_dwconv_wgrad(A, C * H * H, A, C * H * H, A, A, N, C, H, H, K, ws, n, None),
              q, (), (), ("dwconv_wgrad", N, C, H, K))
    for (N, q4, H) in [(16, 16, 128), (16, 64, 32), (2, 8, 64)]:
        if not lib.dsgan_dwconv_multi_supported(H, H, A, 4 * q4 * H * H, A, 4 * q4 * H * H):
            continue
        q = lib.dsgan_dwconv_multi_wgrad_workspace(N, q4, H, H)
        check(lib, lambda ws, n: lib.dsgan_dwconv_multi_wgrad(A, 4 * q4 * H * H, A, 4 * q4 * H * H, A, A, A, A, A, A,
                                                              A, A, N, q4, H, H, ws, n, None),
              q, (), (), ("dwconv_multi", N, q4, H))
    n_split = 0
    for (N, C, HW) in [(16, 3, 65536), (16, 64, 65536), (1, 2, 16384), (2, 5, 20000), (4, 8, 4096)]:
        q = lib.dsgan_instnorm_workspace(N, C, HW)
        n_split += check(lib, lambda ws, n: lib.dsgan_instnorm_fwd_ws(A, C * HW, None, A, C * HW, A, C * HW, A, A, N, C,
                                                                      HW, 1, 0.2, 1e-5, ws, n, None),
                         q, (), (), ("instnorm_fwd", N, C, HW)) > 0
        check(lib, lambda ws, n: lib.dsgan_instnorm_bwd_ws(A, C * HW, A, C * HW, None, None, 0, A, A, A, C * HW, A,
                                                           C * HW, None, N, C, HW, 1, 0.2, 1e-5, ws, n, None),
              q, (), (), ("instnorm_bwd", N, C, HW))
    assert n_split == 3
    check(lib, lambda ws, n: lib.dsgan_ca_bwd(A, A, A, A, A, A, A, A, A, A, A, A, A, 16, 256, 16, ws, n, None),
          16 * (2 * 16 * 256 + 1), (), (), "ca_bwd")
    check(lib, lambda ws, n: lib.dsgan_channel_sum(A, 64 * 1024, A, 16, 64, 1024, ws, n, None), 16 * 64, (), (),
          "channel_sum")
    wts = (ctypes.c_float * 5)(0.0448, 0.2856, 0.3001, 0.2363, 0.1333)
    q = lib.dsgan_ms_ssim_workspace(16, 3, 256, 256)
    check(lib, lambda ws, n: lib.dsgan_ms_ssim(A, A, 0.5, 0.5, 16, 3, 256, 256, A, 1e-4, 9e-4, ctypes.addressof(wts),
                                               5, ws, n, A, A, None), q, (), (), "ms_ssim")
    q = lib.dsgan_ms_ssim_train_workspace(32, 3, 256, 256, 5)
    check(lib, lambda ws, n: lib.dsgan_ms_ssim_fwd_train(A, A, 0.5, 0.5, 32, 3, 256, 256, A, 1e-4, 9e-4,
                                                         ctypes.addressof(wts), 5, ws, n, A, A, None), q, (), (),
          "ms_ssim_fwd_train")
    check(lib, lambda ws, n: lib.dsgan_ms_ssim_bwd(A, A, 0.5, 0.5, 32, 3, 256, 256, A, 1e-4, 9e-4,
                                                   ctypes.addressof(wts), 5, ws, n, A, A, A, 0, None), q, (), (),
          "ms_ssim_bwd")
