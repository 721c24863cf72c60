"""Autograd Functions over libdsgan_hip.so -- the fused ops the DS-GAN networks are built from.

Every forward and backward here is one or more HIP kernels launched on torch's current stream.
PyTorch provides allocation (caching allocator), stream handles and the autograd tape only.

Weight/bias gradients are *accumulated* by the kernels straight into ``param.grad``, which
``dsgan_hip.flat.FlatParams`` binds to a view of one flat fp32 buffer (zeroed once per step);
the Functions therefore return ``None`` for parameters.  A parameter whose ``requires_grad`` is
False (the frozen VGG16, or D during the G step, DSGAN/models/base_model.py:171-177) gets no
weight-grad launch at all.
"""
import contextlib
import os
import math

import ctypes

import torch

from . import _lib
from ._lib import call, ptr, stream


def wsa(t):
    """(pointer, element count) of a scratch tensor (None -> NULL, 0): every scratch-taking entry
    point takes the buffer's size right after it and refuses an undersized one (include/dsgan_hip.h).
    Inside deferred_splits() the tensor is a keep-alive candidate of the call it is passed to: held
    until split_flush() when that call queued a split reduction (which reads it after the call has
    returned), dropped otherwise (InstanceNorm workspaces, forward scratch and the like
    are not held for the whole backward pass)."""
    if t is not None and _DEFER_KEEP[0] is not None:
        _DEFER_CAND.append(t)
    return (ptr(t), t.numel() if t is not None else 0)


# Deferred split reductions (split_reduce.hip): inside deferred_splits() every weight-grad launcher
# queues its fixed-order split reduction (dw += sum_s partials[s]) instead of launching it, and the
# block's end issues the queue as a few batched launches -- ~160 small reduction launches per
# training step become a handful.  Only parameter gradients go through these reductions, and they
# are read only after the backward pass (the optimizer, the non-finite guard) or by the DDP bucket
# all-reduce, which flushes first (dist.GradBuckets._launch).  The scratch of a call that queued a
# reduction (wsa, _keep) is held until the flush.
DEFER_SPLITS = [os.environ.get("DSGAN_DEFER_SPLITS", "1") != "0"]   # (=0: immediate, for A/B runs)
_DEFER_KEEP = [None]
_DEFER_CAND = []


def _defer_hook(queued):
    """_lib.call's report after each entry point: keep that call's candidates if it queued a reduction."""
    if queued and _DEFER_KEEP[0] is not None:
        _DEFER_KEEP[0].extend(_DEFER_CAND)
    _DEFER_CAND.clear()


def _keep(t):
    if _DEFER_KEEP[0] is not None:
        _DEFER_CAND.append(t)
    return t


def split_flush():
    """Launch the queued split reductions (no-op when none are queued)."""
    lib = _lib.load()
    if lib.dsgan_split_pending() > 0:
        call("dsgan_split_flush", stream())
    if _DEFER_KEEP[0] is not None:
        _DEFER_KEEP[0] = []
    _DEFER_CAND.clear()


@contextlib.contextmanager
def deferred_splits():
    """Run a backward pass with its weight-grads' split reductions queued and flushed at the end
    (nested use is a no-op; DEFER_SPLITS[0] = False turns the batching off)."""
    if not DEFER_SPLITS[0] or _DEFER_KEEP[0] is not None:
        yield
        return
    lib = _lib.load()
    _DEFER_KEEP[0] = []
    _DEFER_CAND.clear()
    _lib.DEFER_HOOK[0] = _defer_hook
    lib.dsgan_split_defer(1)
    try:
        yield
    finally:
        lib.dsgan_split_defer(0)
        _lib.DEFER_HOOK[0] = None
        try:
            split_flush()
        finally:
            _DEFER_KEEP[0] = None
            _DEFER_CAND.clear()


# PatchGAN 4x4 weight-grads also sum the conv's bias grad from their staged dy tiles
# (dsgan_wconv_db) instead of a separate channel-sum pass (78 launches per step fewer); the
# round-3 non-finite replay with it does not reproduce on the round-4 tree (tools/nan_diag.py,
# profiles/r04/nan_diag.txt); see DESIGN.md section 6.
WCONV_DB_FOLD = True

ACT = {None: 0, "none": 0, "gelu": 1, "relu": 2, "lrelu": 3, "sigmoid": 4}
ACT_GELU_FAST = 5   # common.h: GELU by A&S 7.1.26 (|err| <= 1.5e-7), the 16-bit modes' InstanceNorm epilogues
PREC = {"fp32": 0, "bf16": 1, "fp16": 1}   # the C ABI's prec: 0 exact f32, 1 16-bit MFMA operands
_state = {"prec": "fp32"}
IN_EPS = 1e-5
LRELU_SLOPE = 0.2


def set_precision(p):
    """'fp32' (exact f32 MFMA, parity mode), 'bf16' (bf16 MFMA operands, fp32 accumulate) or
    'fp16' (IEEE fp16 MFMA operands and 16-bit storage, fp32 accumulate; BASELINE configs[4]).
    bf16 and fp16 run the same kernels: the library's half type (dsgan_set_half_type) selects
    the 16-bit instantiation, so it follows the precision here."""
    if p not in PREC:
        raise ValueError(p)
    _state["prec"] = p
    want = 1 if p == "fp16" else 0
    lib = _lib.load()
    if lib.dsgan_get_half_type() != want:
        call("dsgan_set_half_type", want)


def get_precision():
    return _state["prec"]


@contextlib.contextmanager
def precision(p):
    """Scoped precision: ops created inside run (forward AND backward -- the contraction
    Functions record it in ctx) at precision ``p``.  ``None`` keeps the current one."""
    old = _state["prec"]
    if p is not None:
        set_precision(p)
    try:
        yield
    finally:
        set_precision(old)


def _prec():
    return PREC[_state["prec"]]


def _is16():
    """16-bit MFMA operands (bf16 or fp16 mode)."""
    return _state["prec"] != "fp32"


def half_dtype():
    """torch dtype of the 16-bit operand / storage tensors of the current precision."""
    return torch.float16 if _state["prec"] == "fp16" else torch.bfloat16


class KernelTimer:
    """Brackets every implicit-GEMM launch with HIP events on the launch stream (bench.py's
    roofline leg).  Off by default; when on, records (start, end, algorithmic_flops).

    ``kernel_only=True`` (IGEMM_TIMER) also switches the library's kernel-only timer
    (``dsgan_ktimer``) with it: the pointwise GEMM launchers then record an event pair around the
    GEMM kernel itself, without the split-K finishing pass the same C-ABI call may issue --
    ``pw_kernel_ms()`` reads those, the figure rocprofv3 reports for ``pwgemm_kernel``."""

    def __init__(self, kernel_only=False):
        self._on = False
        self.rec = []
        self.kernel_only = kernel_only

    @property
    def on(self):
        return self._on

    @on.setter
    def on(self, v):
        self._on = bool(v)
        if self.kernel_only:
            _lib.load().dsgan_ktimer(1 if v else 0)

    def reset(self):
        """Drop the records (and the library's kernel-only pairs)."""
        self.rec = []
        if self.kernel_only:
            _lib.load().dsgan_ktimer(-1)

    def pw_kernel_ms(self):
        """Per-launch ms of the pointwise GEMM kernels recorded since reset() (kernel-only timer),
        or None when the library could not read them (events recorded by graph nodes)."""
        lib = _lib.load()
        torch.cuda.synchronize()
        n = lib.dsgan_ktimer(1 if self._on else 0)
        if n <= 0:
            return []
        buf = (ctypes.c_float * n)()
        got = lib.dsgan_ktimer_read(buf, n)
        if got != n:
            return None
        return list(buf)

    def begin(self):
        if not self.on:
            return None
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        return e0

    def end(self, e0, flops, tag=None, fam="other", nbytes=0):
        if e0 is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.rec.append((e0, e1, flops, tag, fam, nbytes))

    def summary(self):
        torch.cuda.synchronize()
        ms = sum(r[0].elapsed_time(r[1]) for r in self.rec)
        fl = sum(r[2] for r in self.rec)
        return dict(launches=len(self.rec), total_ms=ms, flops=fl)

    def families(self):
        """{kernel family: [launches, ms, algorithmic flops, algorithmic bytes]} over the recorded
        launches (bytes: every operand the launch must read or write once, in its stored dtype)."""
        torch.cuda.synchronize()
        out = {}
        for r in self.rec:
            a = out.setdefault(r[4], [0, 0.0, 0.0, 0.0])
            a[0] += 1
            a[1] += r[0].elapsed_time(r[1])
            a[2] += r[2]
            a[3] += r[5]
        return out

    def table(self):
        torch.cuda.synchronize()
        return [(r[0].elapsed_time(r[1]), r[2], r[3] + (r[4],)) for r in self.rec]


IGEMM_TIMER = KernelTimer(kernel_only=True)
AUX_TIMER = KernelTimer()   # the HBM-bound depthwise / InstanceNorm launches (tools/launch_table.py)


def _nb(*ts):
    """HBM bytes of the given operands (None skipped): the algorithmic traffic of a launch."""
    return float(sum(t.numel() * t.element_size() for t in ts if t is not None))


def _conv_flops(N, Cin, Cout, KH, KW, Ho, Wo):
    # algorithmic MACs of the conv (also for its dgrad/wgrad): every output pixel x every tap
    return 2.0 * N * Cout * Cin * KH * KW * Ho * Wo


def _in_act(act):
    """Activation code of an InstanceNorm launch: the 16-bit modes take the A&S GELU (the MLP
    kernels' form); fp32 mode keeps the exact erf."""
    return ACT_GELU_FAST if act == "gelu" and _state["prec"] != "fp32" else ACT[act]


def nchw(t):
    """Return (tensor, batch_stride) with the per-sample [C,H,W] block dense (channel slices of
    a concat buffer qualify); otherwise make it contiguous."""
    if t.dim() != 4:
        raise ValueError("expected NCHW tensor, got %s" % (tuple(t.shape),))
    N, C, H, W = t.shape
    s = t.stride()
    if (s[3] == 1 and s[2] == W and s[1] == H * W) or t.numel() == 0:
        return t, (s[0] if N > 1 else C * H * W)
    t = t.contiguous()
    return t, C * H * W


def _empty(N, C, H, W, like):
    return torch.empty((N, C, H, W), device=like.device, dtype=torch.float32)


# Gradient-readiness hook (dsgan_hip.dist.GradBuckets): every Function calls _params_done() at
# the end of its backward with the parameters whose weight-grads it has just launched, so a
# bucket of the flat gradient can start its all-reduce while the rest of backward runs.
GRAD_READY = [None]


def _params_done(*ps):
    h = GRAD_READY[0]
    if h is not None:
        h([p for p in ps if p is not None])


def _grad_buf(p):
    """Accumulation target for a parameter's gradient, or None when it is frozen."""
    if p is None or not p.requires_grad:
        return None
    if p.grad is None:
        # FlatParams binds .grad up front; a free-standing parameter gets a zeroed buffer here.
        p.grad = torch.zeros_like(p)
    return p.grad


# ------------------------------------------------------------------------------------------
# raw launchers (no autograd)
# ------------------------------------------------------------------------------------------

def _pw_ok(mode, M, K, P, a_bs, b_bs, a, b):
    if not _is16():
        return False
    return bool(_lib.load().dsgan_pw_supported(mode, M, K, P, a_bs, b_bs, a, b))


def _tconv(X, xbs, Wt, bias, Y, ybs, gpre, gbs, nb, K, M, Hin, Win, Hout, Wout, stride, taps,
           Hdst, Wdst, os_, ph, pw, act, gact):
    """Wt: fp32 tap-major weights (_wtrans) or their bf16 copy (_wtrans_bf16, mode 0)."""
    import ctypes
    dh = (ctypes.c_int * len(taps))(*[t[0] for t in taps])
    dw = (ctypes.c_int * len(taps))(*[t[1] for t in taps])
    nws = _lib.load().dsgan_tconv_workspace(nb, K, M, Hout, Wout, len(taps))
    ws = torch.empty(nws, device=X.device, dtype=torch.float32) if nws > 0 else None
    call("dsgan_tconv_ws", ptr(X), xbs, ptr(Wt), ptr(bias), ptr(Y), ybs, ptr(gpre), gbs, nb, K, M, Hin,
         Win, Hout, Wout, stride, len(taps), ctypes.cast(dh, ctypes.c_void_p),
         ctypes.cast(dw, ctypes.c_void_p), Hdst, Wdst, os_, ph, pw, ACT[act], ACT[gact],
         LRELU_SLOPE, int(Wt.dtype != torch.float32), *wsa(ws), stream())


# Transformed-weight cache: an entry is valid while the parameter's storage pointer and the
# global weight generation are unchanged.  FlatAdam.step() bumps the generation (weights are
# updated in place by the fused Adam kernel, invisible to torch's version counters).
WEIGHT_GEN = [0]
_WT_CACHE = {}


_PARAM_GEN = {}


def bump_weight_generation(params=None):
    """Invalidate cached weight transforms: of ``params`` (the ones an optimizer just updated),
    or of every weight.  Frozen weights (VGG16) keep their bf16 / tap-major copies across steps.
    With ``params``, the 16-bit copies cached for them (bf16_weight, _wtrans_bf16) are rebuilt
    right away, in place, by one batched launch (dsgan_wtrans_multi) instead of one launch per
    copy at its next use."""
    if params is None:
        WEIGHT_GEN[0] += 1
    else:
        for p in params:
            _PARAM_GEN[id(p)] = _PARAM_GEN.get(id(p), 0) + 1
        _refresh_half_copies(params)
    if len(_WT_CACHE) > 8192:
        _WT_CACHE.clear()


def _refresh_half_copies(params):
    ids = {id(p) for p in params}
    todo = []   # (cache, key, entry, mode)
    for cache in (_WT_CACHE, _BF16_CACHE):
        for key, ent in cache.items():
            w = ent[2]
            if id(w) not in ids or key[1] != w.data_ptr() or ent[3].dtype == torch.float32:
                continue
            if cache is _WT_CACHE and len(key) != 5:   # (fp32 _wtrans entries are rebuilt lazily)
                continue
            if ent[3].dtype != half_dtype():
                continue
            todo.append((cache, key, ent, key[4] if cache is _WT_CACHE else -1))
    if not todo:
        return
    n = len(todo)
    src = (ctypes.c_void_p * n)(*[e[2][2].data_ptr() for e in todo])
    dst = (ctypes.c_void_p * n)(*[e[2][3].data_ptr() for e in todo])
    desc = []
    for _, _, ent, mode in todo:
        w = ent[2]
        Co, Ci, KH, KW = (tuple(w.shape) + (1, 1, 1))[:4] if w.dim() < 4 else tuple(w.shape)
        if mode < 0:   # plain cast: any shape, as a flat run of numel elements
            Co, Ci, KH, KW = w.numel(), 1, 1, 1
        desc += [Co, Ci, KH, KW, mode]
    dsc = (ctypes.c_int * len(desc))(*desc)
    call("dsgan_wtrans_multi", ctypes.cast(src, ctypes.c_void_p), ctypes.cast(dst, ctypes.c_void_p),
         ctypes.cast(dsc, ctypes.c_void_p), n, stream())
    for cache, key, ent, _ in todo:
        w = ent[2]
        cache[key] = (_wgen(w), w._version, w, ent[3])


def _wgen(w):
    return (WEIGHT_GEN[0], _PARAM_GEN.get(id(w), 0))


def _wtrans(w, mode, kh0=0, kw0=0, nth=0, ntw=0):
    key = (id(w), w.data_ptr(), tuple(w.shape), mode, kh0, kw0, nth, ntw)
    ent = _WT_CACHE.get(key)
    gen = _wgen(w)
    if ent is not None and ent[0] == gen and ent[1] == w._version and ent[2] is w:
        return ent[3]
    wt = _wtrans_build(w, mode, kh0, kw0, nth, ntw)
    _WT_CACHE[key] = (gen, w._version, w, wt)
    return wt


def _wtrans_build(w, mode, kh0=0, kw0=0, nth=0, ntw=0):
    Co, Ci, KH, KW = w.shape
    taps = nth * ntw if mode == 2 else KH * KW
    wt = torch.empty(taps * Co * Ci, device=w.device, dtype=torch.float32)
    call("dsgan_conv_wtrans", ptr(w), ptr(wt), Co, Ci, KH, KW, mode, kh0, kw0, nth, ntw, stream())
    return wt


def _wtrans_bf16(w, mode):
    """bf16 tap-major weights for pconv.hip / pconvt.hip (mode 0 forward, 1 stride-1 data-grad,
    2 stride-2 data-grad / ConvTranspose), cached."""
    key = (id(w), w.data_ptr(), tuple(w.shape), half_dtype(), mode)
    ent = _WT_CACHE.get(key)
    gen = _wgen(w)
    if ent is not None and ent[0] == gen and ent[1] == w._version and ent[2] is w:
        return ent[3]
    Co, Ci, KH, KW = w.shape
    wb = torch.empty(KH * KW * Co * Ci, device=w.device, dtype=half_dtype())
    call("dsgan_conv_wtrans_bf16", ptr(w), ptr(wb), Co, Ci, KH, KW, mode, stream())
    _WT_CACHE[key] = (gen, w._version, w, wb)
    return wb


def _pw_ws(M, N, P, nb, like):
    """Split-K scratch of a pointwise weight-grad (dsgan_pw_wgrad_workspace), or None."""
    n = _lib.load().dsgan_pw_wgrad_workspace(M, N, P, nb)
    return torch.empty(n, device=like.device, dtype=torch.float32) if n > 0 else None


def _pw_io_ok(K, P, xbs, ybs, x, y, pre=None, pbs=0):
    """dsgan_pw_fwd_io / dgrad_io alignment rules with fp32 activations (16-bit weight rows: K % 8)."""
    return (K % 8 == 0 and P % 128 == 0 and xbs % 8 == 0 and ybs % 8 == 0 and x.data_ptr() % 16 == 0
            and y.data_ptr() % 16 == 0 and (pre is None or (pbs % 4 == 0 and pre.data_ptr() % 16 == 0)))


def _pw_fd_ws(mode, M, K, P, nb, like):
    """Split-K scratch of an under-filled pointwise FWD (0) / DGRAD (1) (dsgan_pw_fd_workspace), or None."""
    n = _lib.load().dsgan_pw_fd_workspace(mode, M, K, P, nb)
    return torch.empty(n, device=like.device, dtype=torch.float32) if n > 0 else None


def _pwf_ok(mode, M, K, P, a_bs, b_bs, a, b):
    """fp32 operands (the MidMLKA 1x1 conv, or every 1x1 in the fp32 parity mode): pwf32.hip."""
    return _state["prec"] == "fp32" and bool(_lib.load().dsgan_pw_f32_supported(mode, M, K, P, a_bs, b_bs, a, b))


def _pws_ok(K, M, P, xbs, ybs, x, y):
    """1x1 contraction with <= 16 channels on one side for pwsmall.hip (16-byte rows)."""
    return ((K <= 16 or M <= 16) and x.data_ptr() % 16 == 0 and y.data_ptr() % 16 == 0
            and bool(_lib.load().dsgan_pw_small_supported(K, M, P, xbs, ybs)))


PGLAST = [True]   # the PatchGAN head on pglast.hip (off: the generic small-channel kernels; tests / A-B)


def _pglast_ok(Cout, Cin, KH, KW, stride, pad, H, W, w):
    """Conv(Cin -> 1, 4x4, stride 1, pad 1): the PatchGAN head (networks.py:567-568), pglast.hip."""
    return (PGLAST[0] and Cout == 1 and KH == 4 and KW == 4 and stride == 1 and pad == 1 and w.dim() == 4
            and w.is_contiguous() and bool(_lib.load().dsgan_pglast_supported(Cin, H, W)))


def _thin3_ok(M, H, W, bs_small, bs_big, t_small, t_big):
    """3x3 / s1 / p1 conv with <= 4 channels on one side at W % 256 == 0 (thin3.hip)."""
    return (t_small.data_ptr() % 16 == 0 and t_big.data_ptr() % 16 == 0
            and bool(_lib.load().dsgan_thin3_supported(M, H, W, bs_small, bs_big)))


def _pconv_ok(K, KH, KW, stride):
    return _is16() and bool(_lib.load().dsgan_pconv_supported(K, KH, KW, stride))


def _pconv(x, xbs, wb, b, y, ybs, N, K, M, H, W, Ho, Wo, KH, KW, stride, pad, act, gpre, gbs, gact, accumulate):
    nws = _lib.load().dsgan_pconv_workspace(N, K, M, Ho, Wo)
    ws = torch.empty(nws, device=x.device, dtype=torch.float32) if nws > 0 else None
    call("dsgan_pconv_ws", ptr(x), xbs, ptr(wb), ptr(b), ptr(y), ybs, ptr(gpre), gbs, N, K, M, H, W, Ho, Wo, KH, KW,
         stride, pad, ACT[act], ACT[gact], LRELU_SLOPE, int(accumulate), *wsa(ws), stream())


def conv_fwd_raw(x, w, b, stride, pad, act=None, out=None, pre=None, accumulate=False, xact=None):
    x, xbs = nchw(x)
    N, Cin, H, W = x.shape
    Cout, Cin_w, KH, KW = w.shape if w.dim() == 4 else (w.shape[0], w.shape[1], 1, 1)
    if Cin_w != Cin:
        raise ValueError("conv: input has %d channels, weight expects %d" % (Cin, Cin_w))
    Ho = (H + 2 * pad - KH) // stride + 1
    Wo = (W + 2 * pad - KW) // stride + 1
    y = out if out is not None else _empty(N, Cout, Ho, Wo, x)
    y, ybs = nchw(y)
    pbs = 0
    if pre is not None:
        pre, pbs = nchw(pre)
    e0 = IGEMM_TIMER.begin()
    fam = "igemm_kernel"
    if (KH == 3 and KW == 3 and stride == 1 and pad == 1 and act is None and pre is None and xact is None
            and w.is_contiguous() and _thin3_ok(Cout, H, W, ybs, xbs, y, x)):
        # 3x3 into <= 4 channels at full resolution (the G head): row-strip fp32 stream
        fam = "thin3_kernel"
        call("dsgan_thin3_fwd", ptr(x), xbs, ptr(w), ptr(b), ptr(y), ybs, N, Cin, Cout, H, W, int(accumulate),
             stream())
    elif KH == 1 and KW == 1 and stride == 1 and pad == 0 and pre is None and _pws_ok(Cin, Cout, H * W, xbs, ybs, x, y):
        # 1x1 with <= 16 channels on one side (the 3/12-channel layers at 256^2): VALU stream
        fam = "pw_small_kernel"
        call("dsgan_pw_small", ptr(x), xbs, ptr(w), Cin, 1, ptr(b), ptr(y), ybs, None, 0, N, Cin, Cout, H * W,
             ACT[act], ACT[xact], 0, int(accumulate), LRELU_SLOPE, stream())
    elif _pglast_ok(Cout, Cin, KH, KW, stride, pad, H, W, w) and act is None and pre is None and xact is None:
        # PatchGAN head 256 -> 1, 4x4 s1 (pglast.hip): channel chunks in LDS, partials summed in order
        fam = "pglast_kernel"
        ws = torch.empty(_lib.load().dsgan_pglast_workspace(N, Cin, H, W), device=x.device, dtype=torch.float32)
        call("dsgan_pglast_fwd", ptr(x), xbs, ptr(w), ptr(b), ptr(y), ybs, N, Cin, H, W, int(accumulate), *wsa(ws),
             stream())
    elif Cout <= 8 and act is None and pre is None and xact is None:
        # few output channels (G head, PatchGAN last layer): direct conv, not a GEMM tile
        fam = "small_out_kernel"
        call("dsgan_conv_small_out", ptr(x), xbs, ptr(w), Cin * KH * KW, KH * KW, KW, 1, ptr(b), ptr(y), ybs,
             N, Cin, Cout, H, W, Ho, Wo, KH, KW, stride, pad, 0, int(accumulate), stream())
    elif Cin * KH * KW <= 36 and Cout >= 16 and pre is None and xact is None and act in (None, "relu", "lrelu"):
        # few input taps into many channels (VGG conv1_1): thread-per-pixel exact fp32 dot products
        fam = "small_in_kernel"
        call("dsgan_conv_small_in", ptr(x), xbs, ptr(w), Cin * KH * KW, KH * KW, KW, 1, ptr(b), ptr(y), ybs,
             N, Cin, Cout, H, W, Ho, Wo, KH, KW, stride, pad, 0, ACT[act], LRELU_SLOPE, int(accumulate), stream())
    elif KH == 1 and KW == 1 and stride == 1 and pad == 0 and _pw_ok(0, Cout, Cin, H * W, 0, xbs, w.data_ptr(), x.data_ptr()):
        fam = "pwgemm_kernel"
        if xact is None and _pw_io_ok(Cin, H * W, xbs, ybs, x, y, pre, pbs):
            # the cached 16-bit weight copy instead of converting the fp32 weight tile in every
            # workgroup (the same RNE rounding: the same bits)
            call("dsgan_pw_fwd_io_ws", ptr(bf16_weight(w)), 1, ptr(x), xbs, 0, ptr(y), ybs, 0, ptr(pre), pbs, 0,
                 ptr(b), Cout, Cin, H * W, N, ACT[act], int(accumulate), LRELU_SLOPE,
                 *wsa(_pw_fd_ws(0, Cout, Cin, H * W, N, x)), stream())
        else:
            call("dsgan_pw_gemm", 0, ptr(w), 0, ptr(x), xbs, ptr(y), ybs, ptr(b), ptr(pre), pbs, None, 0,
                 Cout, N * H * W, Cin, H * W, N, ACT[act], 0, ACT[xact], int(accumulate), LRELU_SLOPE,
                 *wsa(_pw_fd_ws(0, Cout, Cin, H * W, N, x)), stream())
    elif (KH == 1 and KW == 1 and stride == 1 and pad == 0 and pre is None and xact is None
          and _pwf_ok(0, Cout, Cin, H * W, 0, xbs, w.data_ptr(), x.data_ptr())):
        fam = "pwf32_kernel"
        call("dsgan_pw_gemm_f32", 0, ptr(w), 0, ptr(x), xbs, ptr(y), ybs, ptr(b), None, 0, Cout, N * H * W, Cin,
             H * W, N, ACT[act], 0, int(accumulate), LRELU_SLOPE, None, 0, stream())
    elif w.dim() == 4 and pre is None and xact is None and _pconv_ok(Cin, KH, KW, stride):
        fam = "pconv_kernel"
        _pconv(x, xbs, _wtrans_bf16(w, 0), b, y, ybs, N, Cin, Cout, H, W, Ho, Wo, KH, KW, stride, pad, act,
               None, 0, None, accumulate)
    elif (_is16() and w.dim() == 4 and (KH > 1 or KW > 1) and Cin % 32 == 0
          and pre is None and not accumulate and xact is None and KH * KW <= 16):
        fam = "tconv_kernel"
        wt = _wtrans_bf16(w, 0) if Cin % 8 == 0 else _wtrans(w, 0)
        taps = [(kh - pad, kw - pad) for kh in range(KH) for kw in range(KW)]
        _tconv(x, xbs, wt, b, y, ybs, None, 0, N, Cin, Cout, H, W, Ho, Wo, stride, taps, Ho, Wo, 1, 0, 0,
               act, None)
    else:
        call("dsgan_conv_fwd", ptr(x), xbs, ptr(w), ptr(b), ptr(y), ybs, ptr(pre), pbs, N, Cin, H, W,
             Cout, KH, KW, stride, pad, Ho, Wo, ACT[act], LRELU_SLOPE, int(accumulate), ACT[xact], _prec(),
             stream())
    IGEMM_TIMER.end(e0, _conv_flops(N, Cin, Cout, KH, KW, Ho, Wo), ("fwd", N, Cin, H, W, Cout, KH, stride), fam,
                    _nb(x, w, b, y, pre) + (_nb(y) if accumulate else 0.0))
    return y


def conv_dgrad_raw(dy, w, x_shape, stride, pad, bias=None, act=None, gpre=None, gact=None,
                   out=None, accumulate=False):
    """dx (N,Cin,H,W) of a conv with weight w [Cout,Cin,KH,KW]; also a ConvTranspose forward."""
    dy, dybs = nchw(dy)
    N, Cin, H, W = x_shape
    Cout, _, KH, KW = w.shape if w.dim() == 4 else (w.shape[0], w.shape[1], 1, 1)
    Ho, Wo = dy.shape[2], dy.shape[3]
    dx = out if out is not None else torch.empty((N, Cin, H, W), device=dy.device, dtype=torch.float32)
    dx, dxbs = nchw(dx)
    gbs = 0
    if gpre is not None:
        gpre, gbs = nchw(gpre)
    e0 = IGEMM_TIMER.begin()
    fam = "igemm_kernel"
    if (KH == 3 and KW == 3 and stride == 1 and pad == 1 and act is None and bias is None and gpre is None
            and w.is_contiguous() and _thin3_ok(Cout, H, W, dybs, dxbs, dy, dx)):
        fam = "thin3_kernel"
        call("dsgan_thin3_dgrad", ptr(dy), dybs, ptr(w), ptr(dx), dxbs, N, Cin, Cout, H, W, int(accumulate), stream())
    elif (KH == 1 and KW == 1 and stride == 1 and pad == 0 and act is None and bias is None
            and _pws_ok(Cout, Cin, H * W, dybs, dxbs, dy, dx) and (gpre is None or (gbs % 4 == 0 and gpre.data_ptr() % 16 == 0))):
        fam = "pw_small_kernel"
        call("dsgan_pw_small", ptr(dy), dybs, ptr(w), 1, Cin, None, ptr(dx), dxbs, ptr(gpre), gbs, N, Cout, Cin, H * W,
             0, 0, ACT[gact], int(accumulate), LRELU_SLOPE, stream())
    elif _pglast_ok(Cout, Cin, KH, KW, stride, pad, H, W, w) and act is None and bias is None and gpre is None:
        fam = "pglast_kernel"
        call("dsgan_pglast_dgrad", ptr(dy), dybs, ptr(w), ptr(dx), dxbs, N, Cin, H, W, int(accumulate), stream())
    elif Cin <= 8 and act is None and gpre is None and stride in (1, 2):
        fam = "small_out_kernel"
        # data-grad into a 3/6-channel tensor: direct transposed gather, w(m=ci, k=co, kh, kw)
        call("dsgan_conv_small_out", ptr(dy), dybs, ptr(w), KH * KW, Cin * KH * KW, KW, 1, ptr(bias),
             ptr(dx), dxbs, N, Cout, Cin, Ho, Wo, H, W, KH, KW, stride, pad, 1, int(accumulate), stream())
    elif Cout * KH * KW <= 27 and KH * KW <= 9 and Cin >= 16 and act is None and gpre is None and stride == 1 and bias is None:
        # data-grad out of a 3-channel conv (G head): stride-1 transposed gather, w(m=ci, k=co, kh, kw)
        fam = "small_in_kernel"
        call("dsgan_conv_small_in", ptr(dy), dybs, ptr(w), KH * KW, Cin * KH * KW, KW, 1, None, ptr(dx), dxbs,
             N, Cout, Cin, Ho, Wo, H, W, KH, KW, 1, pad, 1, 0, LRELU_SLOPE, int(accumulate), stream())
    elif (KH == 1 and KW == 1 and stride == 1 and pad == 0 and bias is None and act is None
            and _pw_ok(1, Cin, Cout, H * W, 0, dybs, w.data_ptr(), dy.data_ptr())):
        fam = "pwgemm_kernel"
        if gpre is None and Cin % 8 == 0 and _pw_io_ok(Cout, H * W, dybs, dxbs, dy, dx):
            call("dsgan_pw_dgrad_io_ws", ptr(bf16_weight(w)), 1, ptr(dy), dybs, 0, ptr(dx), dxbs, 0, None, 0, Cin,
                 Cout, H * W, N, int(accumulate), *wsa(_pw_fd_ws(1, Cin, Cout, H * W, N, dy)), stream())
        else:
            call("dsgan_pw_gemm", 1, ptr(w), 0, ptr(dy), dybs, ptr(dx), dxbs, None, None, 0, ptr(gpre), gbs,
                 Cin, N * H * W, Cout, H * W, N, 0, ACT[gact], 0, int(accumulate), LRELU_SLOPE,
                 *wsa(_pw_fd_ws(1, Cin, Cout, H * W, N, dy)), stream())
    elif (KH == 1 and KW == 1 and stride == 1 and pad == 0 and bias is None and act is None
            and _pwf_ok(1, Cin, Cout, H * W, 0, dybs, w.data_ptr(), dy.data_ptr())):
        fam = "pwf32_kernel"
        call("dsgan_pw_gemm_f32", 1, ptr(w), 0, ptr(dy), dybs, ptr(dx), dxbs, None, ptr(gpre), gbs, Cin, N * H * W,
             Cout, H * W, N, 0, ACT[gact], int(accumulate), LRELU_SLOPE, None, 0, stream())
    elif (w.dim() == 4 and stride == 1 and act is None and bias is None and KH == KW
          and _pconv_ok(Cout, KH, KW, 1)):
        # stride-1 data-grad = forward conv of dy with the flipped, transposed kernel
        fam = "pconv_kernel"
        _pconv(dy, dybs, _wtrans_bf16(w, 1), None, dx, dxbs, N, Cout, Cin, Ho, Wo, H, W, KH, KW, 1,
               KH - 1 - pad, None, gpre, gbs, gact, accumulate)
    elif (_is16() and w.dim() == 4 and stride == 2 and pad == 1 and KH == KW and act is None
          and H <= 2 * Ho and H > 2 * Ho - 2 and W <= 2 * Wo and W > 2 * Wo - 2 and W % 2 == 0 and dxbs % 2 == 0
          and (gpre is None or gbs % 2 == 0) and _lib.load().dsgan_pconvt_supported(Cout, KH, stride, pad)):
        # stride-2 data-grad / ConvTranspose: all four output parities in one launch
        fam = "pconvt_kernel"
        call("dsgan_pconvt", ptr(dy), dybs, ptr(_wtrans_bf16(w, 2)), ptr(bias), ptr(dx), dxbs, ptr(gpre), gbs, N,
             Cout, Cin, Ho, Wo, H, W, KH, stride, pad, ACT[gact], LRELU_SLOPE, int(accumulate), stream())
    elif (_is16() and w.dim() == 4 and (KH > 1 or KW > 1) and Cout % 32 == 0
          and act is None and not accumulate and stride in (1, 2) and KH * KW <= 16):
        fam = "tconv_kernel"
        if stride == 1:
            wt = _wtrans(w, 1)
            pp = KH - 1 - pad
            qq = KW - 1 - pad
            taps = [(kh - pp, kw - qq) for kh in range(KH) for kw in range(KW)]
            _tconv(dy, dybs, wt, bias, dx, dxbs, gpre, gbs, N, Cout, Cin, Ho, Wo, H, W, 1, taps, H, W, 1,
                   0, 0, None, gact)
        else:
            for ph in range(2):
                for pw_ in range(2):
                    kh0, kw0 = (ph + pad) & 1, (pw_ + pad) & 1
                    nth, ntw = (KH - kh0 + 1) // 2, (KW - kw0 + 1) // 2
                    Hc, Wc = (H - ph + 1) // 2, (W - pw_ + 1) // 2
                    if Hc <= 0 or Wc <= 0:
                        continue
                    ch, cw = (ph + pad - kh0) // 2, (pw_ + pad - kw0) // 2
                    wt = _wtrans(w, 2, kh0, kw0, nth, ntw)
                    taps = [(ch - (nth - 1) + a, cw - (ntw - 1) + c) for a in range(nth) for c in range(ntw)]
                    _tconv(dy, dybs, wt, bias, dx, dxbs, gpre, gbs, N, Cout, Cin, Ho, Wo, Hc, Wc, 1, taps,
                           H, W, 2, ph, pw_, None, gact)
    else:
        call("dsgan_conv_dgrad", ptr(dy), dybs, ptr(w), ptr(bias), ptr(dx), dxbs, None, 0, ptr(gpre), gbs,
             ACT[gact], N, Cin, H, W, Cout, KH, KW, stride, pad, Ho, Wo, ACT[act], LRELU_SLOPE,
             int(accumulate), _prec(), stream())
    IGEMM_TIMER.end(e0, _conv_flops(N, Cin, Cout, KH, KW, Ho, Wo), ("dgrad", N, Cin, H, W, Cout, KH, stride), fam,
                    _nb(dy, w, bias, dx, gpre) + (_nb(dx) if accumulate else 0.0))
    return dx


def conv_wgrad_raw(dy, x, dw, stride, pad, xact=None, db=None):
    """dw += conv weight-grad; db (optional) += the bias grad sum(dy) when the kernel taken can fold
    it into the weight-grad (the bf16 pointwise path).  Returns True when db was accumulated."""
    did_db = False
    dy, dybs = nchw(dy)
    x, xbs = nchw(x)
    N, Cin, H, W = x.shape
    Cout = dy.shape[1]
    KH, KW = (dw.shape[2], dw.shape[3]) if dw.dim() == 4 else (1, 1)
    e0 = IGEMM_TIMER.begin()
    fam = "igemm_kernel"
    if (xact is None and KH == 3 and KW == 3 and stride == 1 and pad == 1 and dw.is_contiguous()
            and _thin3_ok(Cout, H, W, dybs, xbs, dy, x)):
        fam = "thin3_kernel"
        ws = torch.empty(_lib.load().dsgan_thin3_wgrad_workspace(N, Cin, Cout, H, W), device=dy.device,
                         dtype=torch.float32)
        call("dsgan_thin3_wgrad", ptr(dy), dybs, ptr(x), xbs, ptr(dw), *wsa(ws), N, Cin, Cout, H, W, stream())
    elif xact is None and dw.is_contiguous() and _pglast_ok(Cout, Cin, KH, KW, stride, pad, H, W, dw):
        fam = "pglast_kernel"
        ws = torch.empty(_lib.load().dsgan_pglast_workspace(N, Cin, H, W), device=dy.device, dtype=torch.float32)
        did_db = db is not None
        call("dsgan_pglast_wgrad", ptr(dy), dybs, ptr(x), xbs, ptr(dw), ptr(db), N, Cin, H, W, *wsa(ws), stream())
    elif xact is None and KH * KW in (1, 9, 16) and (Cout <= 8 or (Cin <= 8 and KH * KW == 1)):
        fam = "wgrad_small_kernel"
        nws = _lib.load().dsgan_conv_wgrad_small_workspace(N, Cin, Cout, KH, KW, dy.shape[2], dy.shape[3])
        ws = torch.empty(nws, device=dy.device, dtype=torch.float32) if nws > 0 else None
        call("dsgan_conv_wgrad_small", ptr(dy), dybs, ptr(x), xbs, ptr(dw), N, Cin, H, W, Cout, KH, KW,
             stride, pad, dy.shape[2], dy.shape[3], *wsa(ws), stream())
    elif KH == 1 and KW == 1 and stride == 1 and pad == 0 and _pw_ok(2, Cout, N * H * W, H * W, dybs, xbs, dy.data_ptr(), x.data_ptr()):
        fam = "pwgemm_kernel"
        did_db = db is not None
        call("dsgan_pw_gemm", 2, ptr(dy), dybs, ptr(x), xbs, ptr(dw), 0, ptr(db), None, 0, None, 0,
             Cout, Cin, N * H * W, H * W, N, 0, 0, ACT[xact], 0, LRELU_SLOPE, *wsa(_pw_ws(Cout, Cin, H * W, N, dy)),
             stream())
    elif (KH == 1 and KW == 1 and stride == 1 and pad == 0 and xact is None
          and _pwf_ok(2, Cout, N * H * W, H * W, dybs, xbs, dy.data_ptr(), x.data_ptr())):
        fam = "pwf32_kernel"
        nws = _lib.load().dsgan_pw_f32_wgrad_workspace(Cout, Cin, H * W, N)
        ws = torch.empty(nws, device=dy.device, dtype=torch.float32) if nws > 0 else None
        did_db = db is not None
        call("dsgan_pw_gemm_f32", 2, ptr(dy), dybs, ptr(x), xbs, ptr(dw), 0, ptr(db), None, 0, Cout, Cin, N * H * W,
             H * W, N, 0, 0, 0, LRELU_SLOPE, *wsa(ws), stream())
    elif (xact is None and _is16() and dw.is_contiguous() and pad == 1 and W % 4 == 0
          and xbs % 4 == 0 and x.data_ptr() % 16 == 0 and _lib.load().dsgan_wconv_supported(Cin, KH, KW, stride)):
        fam = "wconv_kernel"
        Ho, Wo = dy.shape[2], dy.shape[3]
        ws = torch.empty(_lib.load().dsgan_wconv_workspace(N, Cin, Cout, Ho, Wo, KH, KW), device=dy.device,
                         dtype=torch.float32)
        if db is not None and WCONV_DB_FOLD:   # the bias grad from the staged dy tiles (no channel-sum pass)
            did_db = True
            call("dsgan_wconv_db", ptr(dy), dybs, ptr(x), xbs, ptr(dw), ptr(db), *wsa(ws), N, Cin, Cout, H, W, Ho, Wo,
                 KH, KW, stride, pad, stream())
        else:
            call("dsgan_wconv", ptr(dy), dybs, ptr(x), xbs, ptr(dw), *wsa(ws), N, Cin, Cout, H, W, Ho, Wo, KH, KW,
                 stride, pad, stream())
    else:
        nws = _lib.load().dsgan_conv_wgrad_workspace(N, Cin, Cout, KH, KW, dy.shape[2], dy.shape[3], _prec())
        ws = torch.empty(nws, device=dy.device, dtype=torch.float32) if nws > 0 else None
        call("dsgan_conv_wgrad", ptr(dy), dybs, ptr(x), xbs, ptr(dw), N, Cin, H, W, Cout, KH, KW,
             stride, pad, dy.shape[2], dy.shape[3], ACT[xact], _prec(), *wsa(ws), stream())
    IGEMM_TIMER.end(e0, _conv_flops(N, Cin, Cout, KH, KW, dy.shape[2], dy.shape[3]),
                    ("wgrad", N, Cin, H, W, Cout, KH, stride), fam, _nb(dy, x, dw))
    return did_db


def channel_sum_raw(dy, out):
    dy, dybs = nchw(dy)
    N, C, H, W = dy.shape
    ws = torch.empty(N * C, device=dy.device, dtype=torch.float32)
    call("dsgan_channel_sum", ptr(dy), dybs, ptr(out), N, C, H * W, *wsa(ws), stream())


def act_bwd_raw(dy, pre, act, out=None):
    dy = dy.contiguous()
    pre = pre.contiguous()
    out = out if out is not None else torch.empty_like(dy)
    call("dsgan_act_bwd", ptr(dy), ptr(pre), ptr(out), dy.numel(), ACT[act], LRELU_SLOPE, 0, stream())
    return out


def fill_(t, v):
    if not t.is_contiguous():
        raise ValueError("fill_: contiguous tensor required")
    call("dsgan_fill", ptr(t), float(v), t.numel(), stream())
    return t


def zeros(shape, like):
    return fill_(torch.empty(shape, device=like.device, dtype=torch.float32), 0.0)


def copy_multi(pairs):
    """dst <- src for a list of (dst, src) dense fp32 tensors of equal size, one launch per 32 pairs."""
    import ctypes
    if not pairs:
        return
    n = pairs[0][0].numel()
    for d, s in pairs:
        if d.numel() != n or s.numel() != n or not d.is_contiguous() or not s.is_contiguous() \
                or d.dtype != torch.float32 or s.dtype != torch.float32:
            raise ValueError("copy_multi: dense fp32 tensors of one size required")
    srcs = (ctypes.c_void_p * len(pairs))(*[ptr(s) for _, s in pairs])
    dsts = (ctypes.c_void_p * len(pairs))(*[ptr(d) for d, _ in pairs])
    call("dsgan_copy_multi", ctypes.cast(srcs, ctypes.c_void_p), ctypes.cast(dsts, ctypes.c_void_p), len(pairs), n,
         stream())


class CatSlot:
    """The buffer of a channel concatenation cat(head, tail) [N, Ch+Ct, H, W], allocated before
    either half exists.  The tail's producer writes straight into ``tail()`` (a Block output that
    is a decoder skip, MixConvNeXtML.py:229-236), and the node that forms the concatenation
    (ConvTNormFn / InstanceNormCatFn, upSample :61-66) finds the tail already in place and writes
    only the head: the skip is never copied.  ``tail()`` / ``whole()`` alias the buffer's storage
    without being autograd views of it (no kernel writes through torch in-place ops)."""

    def __init__(self, N, Ch, Ct, H, W, like):
        self.buf = _empty(N, Ch + Ct, H, W, like)
        self.Ch, self.Ct = Ch, Ct

    def _alias(self, c0, C):
        b = self.buf
        N, _, H, W = b.shape
        return torch.empty(0, device=b.device, dtype=b.dtype).set_(
            b.untyped_storage(), b.storage_offset() + c0 * H * W, (N, C, H, W), b.stride())

    def tail(self):
        return self._alias(self.Ch, self.Ct)

    def whole(self):
        return self._alias(0, self.Ch + self.Ct)

    def holds(self, t, Ch):
        """t is this slot's tail (behind a head of Ch channels)."""
        b = self.buf
        N, _, H, W = b.shape
        return (t is not None and Ch == self.Ch and t.dim() == 4 and t.dtype == b.dtype and t.device == b.device
                and tuple(t.shape) == (N, self.Ct, H, W) and tuple(t.stride()) == tuple(b.stride())
                and t.data_ptr() == b.data_ptr() + self.Ch * H * W * b.element_size())


def copy_into(dst, src):
    """dst[n] <- src[n] for per-sample dense blocks (used for channel concatenation)."""
    src, sbs = nchw(src)
    dst4, dbs = nchw(dst)
    if dst4.data_ptr() != dst.data_ptr():
        raise ValueError("copy_into: destination must be per-sample dense")
    N = src.shape[0]
    E = src.shape[1] * src.shape[2] * src.shape[3]
    call("dsgan_copy_strided", ptr(src), sbs, ptr(dst), dbs, N, E, stream())


# ------------------------------------------------------------------------------------------
# Shared activations: one gradient buffer per tensor with several consumers.
#
# autograd sums the input-grads of a tensor's consumers with one torch add per extra consumer
# (2 reads + 1 write of the whole tensor each).  ``share(x)`` returns an alias of x carrying a
# _GradBox; consumer Functions see the box on their input and, in backward, either hand their
# freshly computed grad to the box (the first one is adopted as the buffer, no copy) or let the
# kernel accumulate straight into the buffer (maxpool / depthwise / GEMM data-grads have an
# accumulate epilogue).  ShareFn's backward -- run by autograd after every consumer -- returns
# the buffer.  A tensor that may also be referenced elsewhere (a grad autograd handed us) is
# only borrowed, never accumulated into in place.
# ------------------------------------------------------------------------------------------

class _GradBox:
    # outer: the box of the tensor this one aliases (share of a shared tensor, e.g. a Block's input
    # P_i = share(maxpool(R_i))); merged: this box accumulates straight into outer's buffer
    __slots__ = ("buf", "owned", "outer", "merged")

    def __init__(self):
        self.buf, self.owned, self.outer, self.merged = None, False, None, False


def _box(t):
    return getattr(t, "_dsg_box", None)


def _add_n_raw(out, ts):
    import ctypes
    ts4 = [nchw(t) for t in ts]
    o4, obs = nchw(out)
    N, C, H, W = o4.shape
    arr = (ctypes.c_void_p * len(ts4))(*[t.data_ptr() for t, _ in ts4])
    bss = (ctypes.c_long * len(ts4))(*[bs for _, bs in ts4])
    call("dsgan_add_n", ctypes.cast(arr, ctypes.c_void_p), ctypes.cast(bss, ctypes.c_void_p), len(ts4), ptr(o4),
         obs, N, C * H * W, stream())


def _acc_target(box):
    """(buffer, True) when a kernel may accumulate its grad straight into the box.  An empty box
    whose outer box already owns a buffer merges into it: its consumers accumulate into the outer
    buffer in-kernel, instead of filling a buffer of their own that ShareFn then adds to the outer
    one (one add of the whole tensor per nested share)."""
    if box is None:
        return None, False
    if box.buf is None and box.outer is not None:
        ob, _ = _acc_target(box.outer)
        if ob is not None:
            box.buf, box.owned, box.merged = ob, True, True
    if box.buf is not None and box.owned:
        return box.buf, True
    return None, False


def _give(box, t, adopt=True):
    """Route a consumer's input-grad t: returns t itself when the input is not shared."""
    if box is None or t is None:
        return t
    if box.buf is None:
        box.buf, box.owned = t, adopt
    elif box.owned:
        _add_n_raw(box.buf, [box.buf, t])
    else:
        nb = _empty(*t.shape, t)
        _add_n_raw(nb, [box.buf, t])
        box.buf, box.owned = nb, True
    return None


class ShareFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, box):
        ctx.set_materialize_grads(False)
        ctx.box, ctx.outer = box, _box(x)
        box.outer = ctx.outer
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        box = ctx.box
        buf, own, merged = box.buf, box.owned, box.merged
        box.buf, box.merged = None, False
        if g is not None:
            if buf is None:
                buf, own = g, False
            elif own:
                _add_n_raw(buf, [buf, g])
            else:
                nb = _empty(*g.shape, g)
                _add_n_raw(nb, [buf, g])
                buf, own = nb, True
        if merged:
            return None, None   # every grad already sits in the outer box's buffer
        if ctx.outer is not None:
            _give(ctx.outer, buf, adopt=own)
            return None, None
        return buf, None


def share(x):
    """Alias of x whose consumers accumulate into one gradient buffer (see above)."""
    box = _GradBox()
    y = ShareFn.apply(x, box)
    y._dsg_box = box
    return y


# ------------------------------------------------------------------------------------------
# Conv2d (+bias, +relu/lrelu):  VGG 3x3, PatchGAN 4x4, G head 3x3, 1x1 convs
# ------------------------------------------------------------------------------------------

class Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, act):
        y = conv_fwd_raw(x, w, b, stride, pad, act)
        ctx.prec = _state["prec"]
        ctx.stride, ctx.pad, ctx.act = stride, pad, act
        ctx.x_shape = tuple(x.shape)
        ctx.save_for_backward(x, w, b, y if act in ("relu", "lrelu") else None)
        ctx.w_ref, ctx.b_ref = w, b
        ctx.box = _box(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        with precision(ctx.prec):
            return Conv2dFn._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        x, w, b, y = ctx.saved_tensors
        if ctx.act in ("relu", "lrelu"):
            dy = act_bwd_raw(dy, y, ctx.act)  # sign(y) == sign(pre) for relu/lrelu
        dx = None
        if ctx.needs_input_grad[0]:
            out, acc = _acc_target(ctx.box)
            dx = conv_dgrad_raw(dy, w, ctx.x_shape, ctx.stride, ctx.pad, out=out, accumulate=acc)
            dx = None if acc else _give(ctx.box, dx)
        gw = _grad_buf(ctx.w_ref) if ctx.needs_input_grad[1] else None
        gb = _grad_buf(ctx.b_ref) if (b is not None and ctx.needs_input_grad[2]) else None
        if gw is not None and conv_wgrad_raw(dy, x, gw, ctx.stride, ctx.pad, db=gb):
            gb = None
        if gb is not None:
            channel_sum_raw(dy, gb)
        _params_done(ctx.w_ref, ctx.b_ref)
        return dx, None, None, None, None, None


# NLayerDiscriminator layer 0 (networks.py:543-545) on the stem kernels (pgstem.hip); off routes it
# through the generic conv + LeakyReLU backward + bias channel sum (tests, A/B)
PGSTEM = [True]


def _pgstem_ok(x, w, stride, pad, act):
    if not PGSTEM[0] or act != "lrelu" or stride != 2 or pad != 1 or w.dim() != 4 or tuple(w.shape[2:]) != (4, 4):
        return False
    if x.dim() != 4 or not x.is_cuda or not w.is_contiguous() or w.shape[1] != x.shape[1]:
        return False
    N, Cin, H, W = x.shape
    return bool(_lib.load().dsgan_pgstem_supported(Cin, w.shape[0], H, W))


class PatchStemFn(torch.autograd.Function):
    """Conv2d(Cin, ndf, 4, 2, 1) + bias + LeakyReLU(0.2, True), the PatchGAN stem: one kernel per
    direction (dsgan_pgstem_*), exact fp32 in every precision mode.  The backward differentiates
    the LeakyReLU through its saved output, as the reference's in-place activation does."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.box = _box(x)
        x, xbs = nchw(x)
        if xbs % 4 or x.data_ptr() % 16:
            x, xbs = x.contiguous(), x[0].numel()
        N, Cin, H, W = x.shape
        Cout = w.shape[0]
        y = _empty(N, Cout, H // 2, W // 2, x)
        e0 = IGEMM_TIMER.begin()
        call("dsgan_pgstem_fwd", ptr(x), xbs, ptr(w), ptr(b), ptr(y), y[0].numel(), N, Cin, Cout, H, W, LRELU_SLOPE,
             stream())
        IGEMM_TIMER.end(e0, _conv_flops(N, Cin, Cout, 4, 4, H // 2, W // 2), ("fwd", N, Cin, H, W, Cout, 4, 2),
                        "pgstem_kernel", _nb(x, w, b, y))
        ctx.save_for_backward(x, w, b, y)
        ctx.xbs = xbs
        ctx.w_ref, ctx.b_ref = w, b
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, y = ctx.saved_tensors
        dy, dybs = nchw(dy)
        if dybs % 4 or dy.data_ptr() % 16:
            dy, dybs = dy.contiguous(), dy[0].numel()
        N, Cin, H, W = x.shape
        Cout = w.shape[0]
        flops = _conv_flops(N, Cin, Cout, 4, 4, H // 2, W // 2)
        dx = None
        if ctx.needs_input_grad[0]:
            out, acc = _acc_target(ctx.box)
            dx = out if out is not None else _empty(N, Cin, H, W, dy)
            dx4, dxbs = nchw(dx)
            if dx4.data_ptr() != dx.data_ptr():
                raise RuntimeError("PatchStemFn: accumulation target is not NCHW-dense")
            e0 = IGEMM_TIMER.begin()
            call("dsgan_pgstem_dgrad", ptr(dy), dybs, ptr(y), y[0].numel(), ptr(w), ptr(dx), dxbs, N, Cin, Cout, H, W,
                 LRELU_SLOPE, int(acc), stream())
            IGEMM_TIMER.end(e0, flops, ("dgrad", N, Cin, H, W, Cout, 4, 2), "pgstem_kernel",
                            _nb(dy, y, w, dx) + (_nb(dx) if acc else 0.0))
            dx = None if acc else _give(ctx.box, dx)
        gw = _grad_buf(ctx.w_ref) if ctx.needs_input_grad[1] else None
        gb = _grad_buf(ctx.b_ref) if (b is not None and ctx.needs_input_grad[2]) else None
        if gw is not None or gb is not None:
            lib = _lib.load()
            ws = torch.empty(max(lib.dsgan_pgstem_wgrad_workspace(N, Cin, Cout, H, W), 1), device=dy.device,
                             dtype=torch.float32)
            # a frozen weight with a live bias still runs the weight-grad kernel (into scratch)
            dwt = gw if gw is not None else _keep(torch.zeros_like(w))
            e0 = IGEMM_TIMER.begin()
            call("dsgan_pgstem_wgrad", ptr(dy), dybs, ptr(y), y[0].numel(), ptr(x), ctx.xbs, ptr(dwt), ptr(gb), N, Cin,
                 Cout, H, W, LRELU_SLOPE, *wsa(ws), stream())
            IGEMM_TIMER.end(e0, flops, ("wgrad", N, Cin, H, W, Cout, 4, 2), "pgstem_kernel", _nb(dy, y, x, dwt))
        _params_done(ctx.w_ref, ctx.b_ref)
        return dx, None, None


def conv2d(x, w, b=None, stride=1, pad=0, act=None):
    """w may be OIHW or a Linear [out, in] weight (== 1x1 conv); pass the Parameter itself so its
    gradient lands in param.grad."""
    if _pgstem_ok(x, w, stride, pad, act):
        return PatchStemFn.apply(x, w, b)
    return Conv2dFn.apply(x, w, b, stride, pad, act)


# ------------------------------------------------------------------------------------------
# ConvTranspose2d(k3, s2, p1, op1) (+bias): forward = conv data-grad, backward = conv forward
# ------------------------------------------------------------------------------------------

class ConvT3s2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        N, Ci, Hi, Wi = x.shape
        Co = w.shape[1]
        y = conv_dgrad_raw(x, w, (N, Co, 2 * Hi, 2 * Wi), 2, 1, bias=b)
        ctx.prec = _state["prec"]
        ctx.save_for_backward(x, w, b)
        ctx.w_ref, ctx.b_ref = w, b
        ctx.box = _box(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        with precision(ctx.prec):
            return ConvT3s2Fn._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        x, w, b = ctx.saved_tensors
        dx = conv_fwd_raw(dy, w, None, 2, 1) if ctx.needs_input_grad[0] else None
        gw = _grad_buf(ctx.w_ref) if ctx.needs_input_grad[1] else None
        if gw is not None:
            conv_wgrad_raw(x, dy, gw, 2, 1)
        gb = _grad_buf(ctx.b_ref) if (b is not None and ctx.needs_input_grad[2]) else None
        if gb is not None:
            channel_sum_raw(dy, gb)
        _params_done(ctx.w_ref, ctx.b_ref)
        return _give(ctx.box, dx), None, None


def conv_transpose3s2(x, w, b):
    return ConvT3s2Fn.apply(x, w, b)


# ------------------------------------------------------------------------------------------
# ConvNeXt pointwise MLP + shortcut (Block.forward tail, MixConvNeXtML.py:236-242):
#   out = Ws x + W2 gelu(W1 h + b1) + b2
# backward: the dgrad of W2 multiplies by gelu'(z) in its epilogue (no standalone GELU pass).
# ------------------------------------------------------------------------------------------

_BF16_CACHE = {}


def bf16_weight(w):
    """bf16 copy of a parameter for the fused kernels, cached like _wtrans (same invalidation)."""
    key = (id(w), w.data_ptr(), tuple(w.shape), half_dtype())
    ent = _BF16_CACHE.get(key)
    gen = _wgen(w)
    if ent is not None and ent[0] == gen and ent[1] == w._version and ent[2] is w:
        return ent[3]
    out = torch.empty(w.shape, device=w.device, dtype=half_dtype())
    call("dsgan_f32_to_bf16", ptr(w), ptr(out), w.numel(), stream())
    if len(_BF16_CACHE) > 8192:
        _BF16_CACHE.clear()
    _BF16_CACHE[key] = (gen, w._version, w, out)
    return out


def _mlp_tile(C, P, HW, x):
    """Pixels per b1-grad partial row of the fused MLP kernels (mlp.hip), 0 if unsupported."""
    if not _is16() or x.data_ptr() % 16:
        return 0
    return int(_lib.load().dsgan_mlp_supported(C, P, HW))


def _mlp_flops(N, C, P, HW):
    # algorithmic MACs of the two Linear layers (fwd; each of dgrad/wgrad is the same count)
    return 2.0 * N * HW * (4 * C * C + 4 * C * P)


class PwMlpFn(torch.autograd.Function):
    """Block tail: out = Ws x + W2 gelu(W1 h + b1) + b2, h = IN(d) when ``norm`` (the block's
    InstanceNorm, MixConvNeXtML.py:221, folded into this node so that h never needs an fp32 copy).

    In bf16 mode h is stored bf16 (dsgan_instnorm_fwd_bf16): its only readers are bf16-operand
    MFMA GEMMs that round it to bf16 on load anyway, so this halves its bytes and changes no bit.
      * fused shapes (mlp.hip): forward out = Ws x (pwgemm), then out += W2 gelu(W1 h + b1) + b2 in
        one kernel -- z is never stored; backward recomputes z and writes only bf16 gelu(z) and dz
        for the two weight-grads.
      * other bf16 shapes with HW % 128 == 0: pwconv1 evaluates GELU once and writes g = gelu(z) and
        gp = gelu'(z), both bf16; backward writes dz = (W2^T dy) * gp in bf16 (again exactly what
        its two GEMM readers would round to) with the b1 grad summed from the fp32 values in the
        same epilogue.
      * otherwise (fp32 parity mode, tiny shapes) only the pre-GELU hidden z [N,4C,H,W] (fp32) is
        materialised: pwconv2 and its weight-grad read gelu(z) through the GEMM's
        activation-on-load, and the data-grad of pwconv2 multiplies by gelu'(z) in its epilogue."""

    @staticmethod
    def forward(ctx, h, x, w1, b1, w2, b2, ws, norm=False, slot=None, acc=None):
        N, C, H, W = h.shape
        P, HW, C4 = w2.shape[0], H * W, 4 * C
        # out: the slot's tail when the block output is a decoder skip (written in place), or acc
        # itself when the block output is summed into acc (out = acc + block; the first kernel
        # accumulates, acc is returned dirty)
        if acc is not None:
            if (slot is not None or tuple(acc.shape) != (N, P, H, W) or acc.dtype != torch.float32
                    or not acc.is_contiguous()):
                raise ValueError("pw_mlp: acc must be a dense fp32 [%d,%d,%d,%d] tensor (no slot)" % (N, P, H, W))
            ctx.mark_dirty(acc)
        ctx.box_acc = _box(acc) if acc is not None else None
        out0 = slot.tail() if slot is not None else acc
        acc1 = acc is not None
        obs = nchw(out0)[1] if out0 is not None else P * HW
        ctx.refs = (w1, b1, w2, b2, ws)
        ctx.prec = _state["prec"]
        ctx.box_h, ctx.box_x = _box(h), _box(x)
        h, hbs = nchw(h)
        tile = _mlp_tile(C, P, HW, x)
        bigg = (not tile and _is16() and HW % 128 == 0 and C % 8 == 0
                and (norm or h.data_ptr() % 16 == 0))
        ctx.nrm = None
        if norm:
            d, dbs = h, hbs
            if (tile or bigg) and d.data_ptr() % 16 == 0 and dbs % 4 == 0 and HW % 4 == 0:
                mean = torch.empty(N * C, device=d.device, dtype=torch.float32)
                rstd = torch.empty(N * C, device=d.device, dtype=torch.float32)
                h = torch.empty((N, C, H, W), device=d.device, dtype=half_dtype())
                e0 = AUX_TIMER.begin()
                call("dsgan_instnorm_fwd_bf16", ptr(d), dbs, ptr(h), C * HW, ptr(mean), ptr(rstd), N, C, HW, IN_EPS,
                     stream())
                AUX_TIMER.end(e0, 0.0, ("in_fwd_bf16", N, C, H, W), "instnorm", _nb(d, h))
            else:
                h, mean, rstd = instnorm_raw(d)
                tile = tile if h.data_ptr() % 16 == 0 else 0
            hbs = C * HW
            ctx.nrm = (d, mean, rstd)
        elif h.data_ptr() % 16:
            tile = 0
        hb = int(h.dtype != torch.float32)
        ctx.hb = hb
        ctx.tile = tile
        if tile:
            out = conv_fwd_raw(x, ws, None, 1, 0, out=out0, accumulate=acc1)
            e0 = IGEMM_TIMER.begin()
            call("dsgan_mlp_fwd", ptr(h), hbs, hb, ptr(bf16_weight(w1)), ptr(b1), ptr(bf16_weight(w2)), ptr(b2),
                 ptr(out), obs, N, C, P, HW, 1, stream())
            IGEMM_TIMER.end(e0, _mlp_flops(N, C, P, HW), ("mlp_fwd", N, C, H, W, P, 1, 1), "mlp_fwd_kernel",
                            _nb(h, w1, b1, w2, b2) + 2 * _nb(out))
            ctx.save_for_backward(h, x, ws)
            return acc if acc1 else out
        w1v = w1.view(w1.shape[0], w1.shape[1], 1, 1)
        w2v = w2.view(w2.shape[0], w2.shape[1], 1, 1)
        ctx.g = None
        if bigg:
            # large blocks: pwconv1 evaluates GELU once and writes g = gelu(z) and gp = gelu'(z), both
            # bf16; pwconv2 and the W2 weight-grad stream g, the pwconv2 data-grad multiplies by gp
            gp = torch.empty((N, C4, H, W), device=h.device, dtype=half_dtype())   # gelu'(z), for dz
            g = torch.empty((N, C4, H, W), device=h.device, dtype=half_dtype())    # gelu(z)
            e0 = IGEMM_TIMER.begin()
            call("dsgan_pw_fwd_io_ws", ptr(bf16_weight(w1)), 1, ptr(h), hbs, hb, ptr(g), C4 * HW, 1, ptr(gp), C4 * HW, 1,
                 ptr(b1), C4, C, HW, N, ACT["gelu"], 0, LRELU_SLOPE, *wsa(_pw_fd_ws(0, C4, C, HW, N, h)), stream())
            IGEMM_TIMER.end(e0, 2.0 * N * HW * C4 * C, ("fwd", N, C, H, W, C4, 1, 1), "pwgemm_kernel",
                            _nb(h, w1, b1, g, gp))
            out = conv_fwd_raw(x, ws, None, 1, 0, out=out0, accumulate=acc1)
            e0 = IGEMM_TIMER.begin()
            call("dsgan_pw_fwd_io_ws", ptr(bf16_weight(w2)), 1, ptr(g), C4 * HW, 1, ptr(out), obs, 0, None, 0, 0, ptr(b2),
                 P, C4, HW, N, 0, 1, LRELU_SLOPE, *wsa(_pw_fd_ws(0, P, C4, HW, N, g)), stream())
            IGEMM_TIMER.end(e0, 2.0 * N * HW * C4 * P, ("fwd", N, C4, H, W, P, 1, 1), "pwgemm_kernel",
                            _nb(g, w2, b2) + 2 * _nb(out))
            ctx.g = g
            ctx.save_for_backward(h, x, gp, w1v, w2v, ws)
            return acc if acc1 else out
        z = conv_fwd_raw(h, w1v, b1, 1, 0)
        x4, xbs = nchw(x)
        out = out0 if out0 is not None else _empty(N, P, H, W, h)
        if 5 * C <= 16 and _pws_ok(5 * C, P, HW, xbs, obs, x4, z) and z.data_ptr() % 16 == 0 \
                and out.data_ptr() % 16 == 0:
            # tiny blocks (c1: 3 -> 12 -> 64 at 256^2): shortcut + pwconv2 in one streaming pass
            e0 = IGEMM_TIMER.begin()
            call("dsgan_pw_small2", ptr(x4), xbs, ptr(ws), C, 1, ptr(z), 4 * C * HW, ptr(w2), 4 * C, ptr(b2),
                 ptr(out), obs, None, 0, N, C, P, HW, 0, ACT["gelu"], 0, int(acc1), LRELU_SLOPE, stream())
            IGEMM_TIMER.end(e0, 2.0 * N * HW * P * 5 * C, ("fwd", N, 5 * C, H, W, P, 1, 1), "pw_small_kernel",
                            _nb(x4, z, out, ws, w2, b2))
        else:
            conv_fwd_raw(x, ws, None, 1, 0, out=out, accumulate=acc1)
            conv_fwd_raw(z, w2v, b2, 1, 0, out=out, accumulate=True, xact="gelu")
        ctx.save_for_backward(h, x, z, w1v, w2v, ws)
        return acc if acc1 else out

    @staticmethod
    def backward(ctx, dy):
        with precision(ctx.prec):
            if ctx.tile:
                dh, dx = PwMlpFn._backward_fused(ctx, dy)
            else:
                dh, dx = PwMlpFn._backward_unfused(ctx, dy)
            if dh is not None and ctx.nrm is not None:
                d, mean, rstd = ctx.nrm
                dh = instnorm_bwd_raw(dh, d, None, None, mean, rstd, None, False, False)[0]
            ctx.nrm = None
        # out = acc + block: acc's grad is dy itself (borrowed, never adopted as a buffer)
        dacc = _give(ctx.box_acc, dy, adopt=False) if ctx.needs_input_grad[9] else None
        return _give(ctx.box_h, dh), dx, None, None, None, None, None, None, None, dacc

    @staticmethod
    def _backward_unfused(ctx, dy):
        h, x, z, w1v, w2v, ws = ctx.saved_tensors
        w1, b1, w2, b2, ws_ref = ctx.refs
        # dy may be a channel slice of a concat gradient (c1's output feeds the u4 concat): every
        # consumer below takes a batch stride, so only a misaligned slice is copied
        dy, dybs = nchw(dy)
        if dy.data_ptr() % 16 or dybs % 8:
            dy = dy.contiguous()
            dybs = dy.shape[1] * dy.shape[2] * dy.shape[3]
        gw2, gb2, gws, gw1, gb1 = (_grad_buf(t) for t in (w2, b2, ws_ref, w1, b1))
        want_dh = ctx.needs_input_grad[0]
        if ctx.g is not None:
            # bf16 g/gp path (z slot holds gp = gelu'(z)): dz = (W2^T dy) * gp stored bf16, the b1
            # grad as fp32 partial row sums of the same epilogue
            N, C4, H, W = z.shape
            HW, P, C = H * W, w2.shape[0], h.shape[1]
            dz = torch.empty((N, C4, H, W), device=dy.device, dtype=half_dtype())
            e0 = IGEMM_TIMER.begin()
            call("dsgan_pw_dgrad_io_ws", ptr(bf16_weight(w2)), 1, ptr(dy), dybs, 0, ptr(dz), C4 * HW, 1, ptr(z), C4 * HW,
                 C4, P, HW, N, 0, *wsa(_pw_fd_ws(1, C4, P, HW, N, dy)), stream())
            IGEMM_TIMER.end(e0, 2.0 * N * HW * C4 * P, ("dgrad", N, C4, H, W, P, 1, 1), "pwgemm_kernel",
                            _nb(dy, w2, dz, z))
            # bias grads ride on the weight-grads' staged A tiles (db += sum_k A): b2 from dy, b1 from
            # the bf16 dz (as the fused kernels sum it)
            if gw2 is not None:
                e0 = IGEMM_TIMER.begin()
                call("dsgan_pw_wgrad_mixed", ptr(dy), dybs, 0, ptr(ctx.g), C4 * HW, 1, ptr(gw2), ptr(gb2), P, C4,
                     HW, N, *wsa(_pw_ws(P, C4, HW, N, dy)), stream())
                IGEMM_TIMER.end(e0, 2.0 * N * HW * C4 * P, ("wgrad", N, C4, H, W, P, 1, 1), "pwgemm_kernel",
                                _nb(dy, ctx.g, gw2))
            elif gb2 is not None:
                channel_sum_raw(dy, gb2)
            if gws is not None:
                conv_wgrad_raw(dy, x, gws, 1, 0)
            if gw1 is not None:
                e0 = IGEMM_TIMER.begin()
                call("dsgan_pw_wgrad_mixed", ptr(dz), C4 * HW, 1, ptr(h), C * HW, ctx.hb, ptr(gw1), ptr(gb1), C4, C,
                     HW, N, *wsa(_pw_ws(C4, C, HW, N, dz)), stream())
                IGEMM_TIMER.end(e0, 2.0 * N * HW * C4 * C, ("wgrad", N, C, H, W, C4, 1, 1), "pwgemm_kernel",
                                _nb(dz, h, gw1))
            elif gb1 is not None:   # frozen pwconv1 weight, trainable bias (not on the train path)
                channel_sum_raw(dz.float(), gb1)
            dh = None
            if want_dh:
                dh = _empty(N, C, H, W, dy)
                e0 = IGEMM_TIMER.begin()
                call("dsgan_pw_dgrad_io_ws", ptr(bf16_weight(w1)), 1, ptr(dz), C4 * HW, 1, ptr(dh), C * HW, 0, None, 0, C, C4,
                     HW, N, 0, *wsa(_pw_fd_ws(1, C, C4, HW, N, dz)), stream())
                IGEMM_TIMER.end(e0, 2.0 * N * HW * C4 * C, ("dgrad", N, C4, H, W, C, 1, 1), "pwgemm_kernel",
                                _nb(dz, w1, dh))
            _params_done(*ctx.refs)
            return dh, PwMlpFn._dx(ctx, dy, ws, x)
        # fp32 z path: dz = (W2^T dy) * gelu'(z)
        dz = conv_dgrad_raw(dy, w2v, tuple(z.shape), 1, 0, gpre=z, gact="gelu")
        if gw2 is not None and conv_wgrad_raw(dy, z, gw2.view(w2v.shape), 1, 0, xact="gelu", db=gb2):
            gb2 = None
        if gb2 is not None:
            channel_sum_raw(dy, gb2)
        if gws is not None:
            conv_wgrad_raw(dy, x, gws, 1, 0)
        if gw1 is not None and conv_wgrad_raw(dz, h, gw1.view(w1v.shape), 1, 0, db=gb1):
            gb1 = None
        if gb1 is not None:
            channel_sum_raw(dz, gb1)
        dh = conv_dgrad_raw(dz, w1v, tuple(h.shape), 1, 0) if want_dh else None
        _params_done(*ctx.refs)
        return dh, PwMlpFn._dx(ctx, dy, ws, x)

    @staticmethod
    def _dx(ctx, dy, ws, x):
        """shortcut data-grad, accumulated into the shared buffer of x when there is one"""
        if not ctx.needs_input_grad[1]:
            return None
        out, acc = _acc_target(ctx.box_x)
        dx = conv_dgrad_raw(dy, ws, tuple(x.shape), 1, 0, out=out, accumulate=acc)
        return None if acc else _give(ctx.box_x, dx)

    @staticmethod
    def _backward_fused(ctx, dy):
        h, x, ws = ctx.saved_tensors
        w1, b1, w2, b2, ws_ref = ctx.refs
        N, C, H, W = h.shape
        HW, C4, P = H * W, 4 * h.shape[1], w2.shape[0]
        dy, dybs = nchw(dy)
        if dy.data_ptr() % 16:
            dy, dybs = dy.contiguous(), P * HW
        gw2, gb2, gws, gw1, gb1 = (_grad_buf(t) for t in (w2, b2, ws_ref, w1, b1))
        dh = _empty(N, C, H, W, h)
        if gw1 is not None and gb1 is not None and gw2 is not None and C < 256:
            # dh from the data-path kernel; dW1 / db1 / dW2 from the weight-path kernel, which
            # recomputes z and dz per hidden chunk -- gelu(z) and dz never reach HBM.  (Both kernels
            # are GELU/VALU-bound, so the recompute pays only where the bf16 g/dz round trip is the
            # larger cost: measured at B=16, C=128 @256^2 1.98 -> 1.77 ms, C=256 @128^2 1.70 -> 1.94 ms.)
            w1b, w2b = bf16_weight(w1), bf16_weight(w2)
            e0 = IGEMM_TIMER.begin()
            call("dsgan_mlp_bwd", ptr(h), C * HW, ctx.hb, ptr(dy), dybs, ptr(w1b), ptr(b1), ptr(w2b), ptr(dh), C * HW,
                 None, None, None, N, C, P, HW, stream())
            IGEMM_TIMER.end(e0, 2.0 * N * HW * C4 * (2 * C + P), ("mlp_bwd", N, C, H, W, P, 1, 1), "mlp_bwd_kernel",
                            _nb(h, dy, w1, b1, w2, dh))
            wsp = torch.empty(_lib.load().dsgan_mlp_wgrad_workspace(C, P, HW, N), device=h.device, dtype=torch.float32)
            e0 = IGEMM_TIMER.begin()
            call("dsgan_mlp_wgrad", ptr(h), C * HW, ctx.hb, ptr(dy), dybs, ptr(w1b), ptr(b1), ptr(w2b), ptr(gw1),
                 ptr(gb1), ptr(gw2), *wsa(wsp), N, C, P, HW, stream())
            IGEMM_TIMER.end(e0, 2.0 * N * HW * C4 * (2 * C + 2 * P), ("mlp_wgrad", N, C, H, W, P, 1, 1),
                            "mlp_wgrad_kernel", _nb(h, dy, w1, b1, w2, gw1, gb1, gw2))
            if gb2 is not None:
                channel_sum_raw(dy, gb2)
            if gws is not None:
                conv_wgrad_raw(dy, x, gws, 1, 0)
            _params_done(*ctx.refs)
            return dh, PwMlpFn._dx(ctx, dy, ws, x)
        g = torch.empty((N, C4, H, W), device=h.device, dtype=half_dtype())
        dz = torch.empty_like(g)
        e0 = IGEMM_TIMER.begin()
        call("dsgan_mlp_bwd", ptr(h), C * HW, ctx.hb, ptr(dy), dybs, ptr(bf16_weight(w1)), ptr(b1),
             ptr(bf16_weight(w2)), ptr(dh), C * HW, ptr(g), ptr(dz), None, N, C, P, HW, stream())
        IGEMM_TIMER.end(e0, _mlp_flops(N, C, P, HW), ("mlp_bwd", N, C, H, W, P, 1, 1), "mlp_bwd_kernel",
                        _nb(h, dy, w1, b1, w2, dh, g, dz))
        # bias grads from the weight-grads' staged A tiles: b2 = sum dy, b1 = sum of the bf16 dz
        if gw2 is not None:
            e0 = IGEMM_TIMER.begin()
            call("dsgan_pw_wgrad_mixed", ptr(dy), dybs, 0, ptr(g), C4 * HW, 1, ptr(gw2), ptr(gb2), P, C4, HW, N,
                 *wsa(_pw_ws(P, C4, HW, N, dy)), stream())
            IGEMM_TIMER.end(e0, 2.0 * N * HW * C4 * P, ("wgrad", N, C4, H, W, P, 1, 1), "pwgemm_kernel",
                            _nb(dy, g, gw2))
        elif gb2 is not None:
            channel_sum_raw(dy, gb2)
        if gws is not None:
            conv_wgrad_raw(dy, x, gws, 1, 0)
        if gw1 is not None:
            e0 = IGEMM_TIMER.begin()
            call("dsgan_pw_wgrad_mixed", ptr(dz), C4 * HW, 1, ptr(h), C * HW, ctx.hb, ptr(gw1), ptr(gb1), C4, C, HW,
                 N, *wsa(_pw_ws(C4, C, HW, N, dz)), stream())
            IGEMM_TIMER.end(e0, 2.0 * N * HW * C4 * C, ("wgrad", N, C, H, W, C4, 1, 1), "pwgemm_kernel",
                            _nb(dz, h, gw1))
        elif gb1 is not None:
            channel_sum_raw(dz.float(), gb1)
        _params_done(*ctx.refs)
        return dh, PwMlpFn._dx(ctx, dy, ws, x)


def pw_mlp(h, x, w1, b1, w2, b2, ws, norm=False, slot=None, acc=None):
    """ConvNeXt block tail; with norm=True the first argument is the depthwise-conv output d and
    the block's InstanceNorm h = IN(d) is applied inside (MixConvNeXtML.py:219-224).  ``slot``
    (CatSlot): the output is written into the slot's tail and returned as that alias.  ``acc``: the
    output is summed into acc in place (acc + block, the shortcut GEMM's epilogue adds acc) and acc
    is returned."""
    return PwMlpFn.apply(h, x, w1, b1, w2, b2, ws, norm, slot, acc)


# ------------------------------------------------------------------------------------------
# Depthwise conv
# ------------------------------------------------------------------------------------------

def dwconv_raw(x, w, b, flip=False, out=None, accumulate=False):
    x, xbs = nchw(x)
    N, C, H, W = x.shape
    K = w.shape[-1]
    y = out if out is not None else _empty(N, C, H, W, x)
    y4, ybs = nchw(y)
    e0 = AUX_TIMER.begin()
    call("dsgan_dwconv_fwd", ptr(x), xbs, ptr(w), ptr(b), ptr(y4), ybs, N, C, H, W, K, int(flip), int(accumulate),
         stream())
    AUX_TIMER.end(e0, 2.0 * N * C * H * W * K * K, ("dw_dgrad" if flip else "dw_fwd", N, C, H, W, K), "dwconv",
                  (3 if accumulate else 2) * _nb(x))
    return y4


def _dw_wgrad(dy, x, gw, gb, K):
    dy4, dybs = nchw(dy)
    x4, xbs = nchw(x)
    N, C, H, W = x4.shape
    al = int(x4.data_ptr() % 16 == 0 and dy4.data_ptr() % 16 == 0 and xbs % 4 == 0 and dybs % 4 == 0)
    ws = torch.empty(_lib.load().dsgan_dwconv_wgrad_workspace(N, C, H, W, K, al), device=x4.device, dtype=torch.float32)
    e0 = AUX_TIMER.begin()
    call("dsgan_dwconv_wgrad", ptr(dy4), dybs, ptr(x4), xbs, ptr(gw), ptr(gb), N, C, H, W, K, *wsa(ws), stream())
    AUX_TIMER.end(e0, 2.0 * N * C * H * W * K * K, ("dw_wgrad", N, C, H, W, K), "dwconv", 2 * _nb(x4))


class DwConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        y = dwconv_raw(x, w, b)
        ctx.save_for_backward(x, w)
        ctx.refs = (w, b)
        ctx.box = _box(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        wr, br = ctx.refs
        dx = None
        if ctx.needs_input_grad[0]:
            out, acc = _acc_target(ctx.box)
            dx = dwconv_raw(dy, w, None, flip=True, out=out, accumulate=acc)
            dx = None if acc else _give(ctx.box, dx)
        gw, gb = _grad_buf(wr), _grad_buf(br)
        if gw is not None:
            _dw_wgrad(dy, x, gw, gb, w.shape[-1])
        _params_done(wr, br)
        return dx, None, None


def dwconv(x, w, b):
    return DwConvFn.apply(x, w, b)


class MultiDwConvFn(torch.autograd.Function):
    """MidMLKA's chunk(4) -> X3/X5/X7/X9 depthwise -> cat (MixConvNeXtML.py:110-111), written
    straight into one output buffer (no chunk/cat copies); one launch per pass over the four
    quarters where the plane shape takes a tiled configuration (dsgan_dwconv_multi_*)."""

    @staticmethod
    def _multi_ok(x4, xbs, y, ybs):
        N, C, H, W = x4.shape
        return C % 4 == 0 and bool(_lib.load().dsgan_dwconv_multi_supported(H, W, ptr(x4), xbs, ptr(y), ybs))

    @staticmethod
    def forward(ctx, x, *wb):
        x4, xbs = nchw(x)
        N, C, H, W = x4.shape
        q = C // 4
        y = _empty(N, C, H, W, x4)
        if MultiDwConvFn._multi_ok(x4, xbs, y, C * H * W):
            e0 = AUX_TIMER.begin()
            call("dsgan_dwconv_multi_fwd", ptr(x4), xbs, *[ptr(t) for t in wb], ptr(y), C * H * W, N, q, H, W, 0, 0,
                 stream())
            AUX_TIMER.end(e0, 2.0 * N * q * H * W * (9 + 25 + 49 + 81), ("dw_multi_fwd", N, C, H, W, 0), "dwconv",
                          2 * _nb(x4))
        else:
            for i in range(4):
                dwconv_raw(x4[:, i * q:(i + 1) * q], wb[2 * i], wb[2 * i + 1], out=y[:, i * q:(i + 1) * q])
        ctx.save_for_backward(x4, *wb)
        ctx.refs = wb
        ctx.box = _box(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, *wb = ctx.saved_tensors
        N, C, H, W = x.shape
        q = C // 4
        dy4, dybs = nchw(dy)
        out, acc = _acc_target(ctx.box)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = out if acc else _empty(N, C, H, W, x)
        grads = [_grad_buf(r) for r in ctx.refs]
        xbs = x.stride(0) if N > 1 else C * H * W
        multi = MultiDwConvFn._multi_ok(x, xbs, dy4, dybs) and (dx is None or dx.stride(0) == C * H * W or N == 1)
        if multi:
            if dx is not None:
                e0 = AUX_TIMER.begin()
                call("dsgan_dwconv_multi_fwd", ptr(dy4), dybs, *[ptr(t) if i % 2 == 0 else None for i, t in enumerate(wb)],
                     ptr(dx), C * H * W, N, q, H, W, 1, int(acc), stream())
                AUX_TIMER.end(e0, 2.0 * N * q * H * W * 164, ("dw_multi_dgrad", N, C, H, W, 0), "dwconv",
                              (3 if acc else 2) * _nb(x))
            if all(g_ is not None for g_ in grads):
                wsp = torch.empty(_lib.load().dsgan_dwconv_multi_wgrad_workspace(N, q, H, W), device=x.device,
                                  dtype=torch.float32)
                e0 = AUX_TIMER.begin()
                call("dsgan_dwconv_multi_wgrad", ptr(dy4), dybs, ptr(x), xbs, *[ptr(g_) for g_ in grads], N, q, H, W,
                     *wsa(wsp), stream())
                AUX_TIMER.end(e0, 2.0 * N * q * H * W * 164, ("dw_multi_wgrad", N, C, H, W, 0), "dwconv", 2 * _nb(x))
                grads = [None] * 8
        else:
            for i in range(4):
                sl = slice(i * q, (i + 1) * q)
                if dx is not None:
                    dwconv_raw(dy4[:, sl], wb[2 * i], None, flip=True, out=dx[:, sl], accumulate=acc)
        for i in range(4):
            gw, gb = grads[2 * i], grads[2 * i + 1]
            if gw is not None:
                sl = slice(i * q, (i + 1) * q)
                _dw_wgrad(dy4[:, sl], x[:, sl], gw, gb, wb[2 * i].shape[-1])
        dx = None if acc else _give(ctx.box, dx)
        _params_done(*ctx.refs)
        return (dx,) + (None,) * 8


def multi_dwconv(x, w3, b3, w5, b5, w7, b7, w9, b9):
    return MultiDwConvFn.apply(x, w3, b3, w5, b5, w7, b7, w9, b9)


# ------------------------------------------------------------------------------------------
# InstanceNorm (+scale, +residual, +act)
# ------------------------------------------------------------------------------------------

def _in_ws(N, C, HW, like):
    """Scratch of the split InstanceNorm forms (few large planes), None when the shape needs none."""
    n = _lib.load().dsgan_instnorm_workspace(N, C, HW)
    return torch.empty(n, device=like.device, dtype=torch.float32) if n > 0 else None


def instnorm_raw(x, scale=None, res=None, act=None, out=None):
    x, xbs = nchw(x)
    N, C, H, W = x.shape
    rbs = 0
    if res is not None:
        res, rbs = nchw(res)
    y = out if out is not None else _empty(N, C, H, W, x)
    y4, ybs = nchw(y)
    mean = torch.empty(N * C, device=x.device, dtype=torch.float32)
    rstd = torch.empty(N * C, device=x.device, dtype=torch.float32)
    e0 = AUX_TIMER.begin()
    call("dsgan_instnorm_fwd_ws", ptr(x), xbs, ptr(scale), ptr(res), rbs, ptr(y4), ybs, ptr(mean),
         ptr(rstd), N, C, H * W, _in_act(act), LRELU_SLOPE, IN_EPS, *wsa(_in_ws(N, C, H * W, x)), stream())
    AUX_TIMER.end(e0, 0.0, ("in_fwd", N, C, H, W, act, res is not None), "instnorm", (3 if res is not None else 2) * _nb(x))
    return y4, mean, rstd


def instnorm_bwd_raw(dy, x, scale, res, mean, rstd, act, want_dres, want_dscale):
    dy, dybs = nchw(dy)
    x, xbs = nchw(x)
    N, C, H, W = x.shape
    rbs = 0
    if res is not None:
        res, rbs = nchw(res)
    dx = _empty(N, C, H, W, x)
    dres = _empty(N, C, H, W, x) if want_dres else None
    dscale = torch.empty(N * C, device=x.device, dtype=torch.float32) if want_dscale else None
    e0 = AUX_TIMER.begin()
    call("dsgan_instnorm_bwd_ws", ptr(dy), dybs, ptr(x), xbs, ptr(scale), ptr(res), rbs, ptr(mean),
         ptr(rstd), ptr(dx), C * H * W, ptr(dres), C * H * W, ptr(dscale), N, C, H * W, _in_act(act),
         LRELU_SLOPE, IN_EPS, *wsa(_in_ws(N, C, H * W, x)), stream())
    AUX_TIMER.end(e0, 0.0, ("in_bwd", N, C, H, W, act, res is not None), "instnorm",
                  (3 + (res is not None) + want_dres) * _nb(x))
    return dx, dres, dscale


class InstanceNormFn(torch.autograd.Function):
    """y = act(IN(x) + res) -- InstanceNorm2d(affine=False) fused with what follows it."""

    @staticmethod
    def forward(ctx, x, res, act):
        y, mean, rstd = instnorm_raw(x, None, res, act)
        ctx.act = act
        ctx.save_for_backward(x, res, mean, rstd)
        ctx.box_x, ctx.box_r = _box(x), (_box(res) if res is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, res, mean, rstd = ctx.saved_tensors
        dx, dres, _ = instnorm_bwd_raw(dy, x, None, res, mean, rstd, ctx.act,
                                       res is not None and ctx.needs_input_grad[1], False)
        return _give(ctx.box_x, dx), _give(ctx.box_r, dres), None


def instance_norm(x, act=None, res=None):
    return InstanceNormFn.apply(x, res, act)


class InstanceNormCatFn(torch.autograd.Function):
    """cat(act(IN(x)), skip) along channels: the IN kernel writes its plane straight into the
    first Ca channels of the concatenation (upSample, MixConvNeXtML.py:61-66), so only the skip
    is copied; the backward reads its slice of dy in place."""

    @staticmethod
    def forward(ctx, x, skip, act, slot=None):
        N, Ca, H, W = x.shape
        if slot is not None and slot.holds(skip, Ca):
            out = slot.whole()   # the skip's producer already wrote it into the tail
            _, mean, rstd = instnorm_raw(x, None, None, act, out=out[:, :Ca])
        else:
            out = _empty(N, Ca + skip.shape[1], H, W, x)
            _, mean, rstd = instnorm_raw(x, None, None, act, out=out[:, :Ca])
            copy_into(out[:, Ca:], skip)
        ctx.act, ctx.Ca = act, Ca
        ctx.save_for_backward(x, mean, rstd)
        ctx.box_x, ctx.box_s = _box(x), _box(skip)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd = ctx.saved_tensors
        dx, _, _ = instnorm_bwd_raw(dy[:, :ctx.Ca], x, None, None, mean, rstd, ctx.act, False, False)
        return _give(ctx.box_x, dx), _give(ctx.box_s, dy[:, ctx.Ca:]), None, None


def instance_norm_cat(x, skip, act=None, slot=None):
    return InstanceNormCatFn.apply(x, skip, act, slot)


class ConvTNormFn(torch.autograd.Function):
    """ConvTranspose2d 3x3/s2 (pad 1, output_padding 1) feeding the decoder InstanceNorm:
    cat(act(IN(convT(x))), skip) (upSample, MixConvNeXtML.py:48-66) or act(IN(convT(x)) + res)
    (OriginMLKA tail, :150-152).  The forward is ConvT3s2Fn's then InstanceNorm(Cat)Fn's.  The
    backward keeps the ConvT output grad off fp32: dsgan_instnorm_bwd_h stores it in the 16-bit
    half type with its per-plane sums, the ConvT data-grad (dsgan_tconv_ws_xh) and weight-grad
    (dsgan_wconv_xh) read those 16 bits as MFMA operands -- exactly the values the fp32-input forms
    round to on load, so dx and dW are unchanged -- and the bias grad is the sum over images of
    the plane sums (the fp32 values, as channel_sum of the fp32 grad would add them)."""

    @staticmethod
    def forward(ctx, x, w, b, other, act, cat, slot=None):
        N, Ci, Hi, Wi = x.shape
        Co = w.shape[1]
        t = conv_dgrad_raw(x, w, (N, Co, 2 * Hi, 2 * Wi), 2, 1, bias=b)
        if cat:
            if slot is not None and slot.holds(other, Co):
                out = slot.whole()   # the skip's producer already wrote it into the tail
                _, mean, rstd = instnorm_raw(t, None, None, act, out=out[:, :Co])
            else:
                out = _empty(N, Co + other.shape[1], 2 * Hi, 2 * Wi, t)
                _, mean, rstd = instnorm_raw(t, None, None, act, out=out[:, :Co])
                copy_into(out[:, Co:], other)
            ctx.save_for_backward(x, w, t, mean, rstd)
        else:
            out, mean, rstd = instnorm_raw(t, None, other, act)
            ctx.save_for_backward(x, w, t, mean, rstd, other)
        ctx.prec, ctx.act, ctx.cat, ctx.has_b = _state["prec"], act, cat, b is not None
        ctx.w_ref, ctx.b_ref = w, b
        ctx.box_x, ctx.box_o = _box(x), _box(other)
        return out

    @staticmethod
    def backward(ctx, dy):
        with precision(ctx.prec):
            return ConvTNormFn._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        import ctypes
        if ctx.cat:
            x, w, t, mean, rstd = ctx.saved_tensors
            res = None
        else:
            x, w, t, mean, rstd, res = ctx.saved_tensors
        N, Ci, Hi, Wi = x.shape
        Co, H, W = t.shape[1], t.shape[2], t.shape[3]
        HW = H * W
        dyt, dybs = nchw(dy[:, :Co] if ctx.cat else dy)
        t4, tbs = nchw(t)
        rbs = 0
        if res is not None:
            res, rbs = nchw(res)
        want_dres = res is not None and ctx.needs_input_grad[3]
        dres = _empty(N, Co, H, W, t) if want_dres else None
        dth = torch.empty((N, Co, H, W), device=t.device, dtype=half_dtype())
        psum = torch.empty(N * Co, device=t.device, dtype=torch.float32)
        e0 = AUX_TIMER.begin()
        call("dsgan_instnorm_bwd_h", ptr(dyt), dybs, ptr(t4), tbs, ptr(res), rbs, ptr(mean), ptr(rstd), ptr(dth),
             Co * HW, ptr(psum), ptr(dres), Co * HW, N, Co, HW, _in_act(ctx.act), LRELU_SLOPE, IN_EPS, stream())
        AUX_TIMER.end(e0, 0.0, ("in_bwd_h", N, Co, H, W, ctx.act, res is not None), "instnorm",
                      _nb(dyt, t4, res, dres) + _nb(dth))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _empty(N, Ci, Hi, Wi, x)
            taps = [(kh - 1, kw - 1) for kh in range(3) for kw in range(3)]
            dh = (ctypes.c_int * 9)(*[q[0] for q in taps])
            dw = (ctypes.c_int * 9)(*[q[1] for q in taps])
            nws = _lib.load().dsgan_tconv_workspace(N, Co, Ci, Hi, Wi, 9)
            ws = torch.empty(nws, device=t.device, dtype=torch.float32) if nws > 0 else None
            e0 = IGEMM_TIMER.begin()
            call("dsgan_tconv_ws_xh", ptr(dth), Co * HW, ptr(_wtrans_bf16(w, 0)), None, ptr(dx), Ci * Hi * Wi, None,
                 0, N, Co, Ci, H, W, Hi, Wi, 2, 9, ctypes.cast(dh, ctypes.c_void_p), ctypes.cast(dw, ctypes.c_void_p),
                 Hi, Wi, 1, 0, 0, 0, 0, LRELU_SLOPE, *wsa(ws), stream())
            IGEMM_TIMER.end(e0, _conv_flops(N, Co, Ci, 3, 3, Hi, Wi), ("fwd", N, Co, H, W, Ci, 3, 2), "tconv_kernel",
                            _nb(dth, dx) + 2.0 * w.numel())
        gw = _grad_buf(ctx.w_ref) if ctx.needs_input_grad[1] else None
        if gw is not None:
            x4, xbs = nchw(x)
            ws = torch.empty(_lib.load().dsgan_wconv_workspace(N, Co, Ci, Hi, Wi, 3, 3), device=t.device,
                             dtype=torch.float32)
            e0 = IGEMM_TIMER.begin()
            call("dsgan_wconv_xh", ptr(x4), xbs, ptr(dth), Co * HW, ptr(gw), *wsa(ws), N, Co, Ci, H, W, Hi, Wi, 3, 3,
                 2, 1, stream())
            IGEMM_TIMER.end(e0, _conv_flops(N, Co, Ci, 3, 3, Hi, Wi), ("wgrad", N, Co, H, W, Ci, 3, 2), "wconv_kernel",
                            _nb(x4, dth, gw))
        gb = _grad_buf(ctx.b_ref) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        if gb is not None:
            channel_sum_raw(psum.view(N, Co, 1, 1), gb)
        _params_done(ctx.w_ref, ctx.b_ref)
        dother = _give(ctx.box_o, dy[:, Co:]) if ctx.cat else _give(ctx.box_o, dres)
        return _give(ctx.box_x, dx), None, None, dother, None, None, None


def _convt_norm_fused(x, w, other, cat):
    """The fused ConvT + InstanceNorm backward's conditions: 16-bit operands (bf16 / fp16 mode),
    K (ConvT output channels) % 32 for the 16-bit-operand kernels, float4-aligned planes."""
    N, Ci, Hi, Wi = x.shape
    Co = w.shape[1]
    HW = 4 * Hi * Wi
    return (_is16() and w.dim() == 4 and w.shape[2] == 3 and w.shape[3] == 3 and Co % 32 == 0 and Ci % 32 == 0
            and HW % 4 == 0 and (2 * Wi) % 4 == 0 and bool(_lib.load().dsgan_wconv_supported(Co, 3, 3, 2)))


def convt_norm(x, w, b, other, act=None, cat=False, slot=None):
    """cat(act(IN(ConvT3s2(x))), other) if cat else act(IN(ConvT3s2(x)) + other) (other may be None).
    ``slot`` (CatSlot, cat only): when ``other`` is the slot's tail the concatenation is formed in
    place and returned as ``slot.whole()``."""
    if _convt_norm_fused(x, w, other, cat):
        return ConvTNormFn.apply(x, w, b, other, act, cat, slot)
    y = conv_transpose3s2(x, w, b)
    return instance_norm_cat(y, other, act, slot) if cat else instance_norm(y, act, other)


# ------------------------------------------------------------------------------------------
# MaxPool2d(k) with int32 plane-flat argmax
# ------------------------------------------------------------------------------------------

class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k):
        x4, xbs = nchw(x)
        N, C, H, W = x4.shape
        Ho, Wo = H // k, W // k
        y = _empty(N, C, Ho, Wo, x4)
        idx = torch.empty((N, C, Ho, Wo), device=x4.device, dtype=torch.int32)
        call("dsgan_maxpool_fwd", ptr(x4), xbs, ptr(y), C * Ho * Wo, ptr(idx), N, C, H, W, k, stream())
        ctx.k, ctx.shape = k, (N, C, H, W)
        ctx.save_for_backward(idx)
        ctx.mark_non_differentiable(idx)
        # (no zero-filled int grad for idx per backward: autograd would materialise one)
        ctx.set_materialize_grads(False)
        ctx.box = _box(x)
        return y, idx

    @staticmethod
    def backward(ctx, dy, _didx):
        if dy is None:
            return None, None
        (idx,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        dy4, dybs = nchw(dy)
        out, acc = _acc_target(ctx.box)
        dx = out if acc else torch.empty((N, C, H, W), device=dy.device, dtype=torch.float32)
        dx4, dxbs = nchw(dx)
        if dx4.data_ptr() != dx.data_ptr():
            raise RuntimeError("maxpool backward: gradient buffer must be per-sample dense")
        call("dsgan_maxpool_bwd", ptr(dy4), dybs, ptr(idx), ptr(dx4), dxbs, N, C, H, W, ctx.k, int(acc), stream())
        return (None if acc else _give(ctx.box, dx)), None


class MaxPoolPyrFn(torch.autograd.Function):
    """MaxPool2d(2), (4), ... (2^levels) of one tensor (the skip pyramids) in one launch each way
    (dsgan_maxpool_pyr_*): one read of x instead of one per k, and one read-modify-write of its
    gradient instead of one per k."""

    @staticmethod
    def forward(ctx, x, levels):
        x4, xbs = nchw(x)
        N, C, H, W = x4.shape
        ys, ids = [], []
        for lv in range(levels):
            k = 2 << lv
            ys.append(_empty(N, C, H // k, W // k, x4))
            ids.append(torch.empty((N, C, H // k, W // k), device=x4.device, dtype=torch.int32))
        args = []
        for lv in range(4):
            args += [ptr(ys[lv]), ptr(ids[lv])] if lv < levels else [None, None]
        call("dsgan_maxpool_pyr_fwd", ptr(x4), xbs, levels, *args, N, C, H, W, stream())
        ctx.levels, ctx.shape = levels, (N, C, H, W)
        ctx.save_for_backward(*ids)
        ctx.mark_non_differentiable(*ids)
        ctx.set_materialize_grads(False)
        ctx.box = _box(x)
        return tuple(ys) + tuple(ids)

    @staticmethod
    def backward(ctx, *grads):
        L = ctx.levels
        dys = grads[:L]
        if all(g is None for g in dys):
            return None, None
        ids = ctx.saved_tensors
        N, C, H, W = ctx.shape
        out, acc = _acc_target(ctx.box)
        dx = out if acc else torch.empty((N, C, H, W), device=ids[0].device, dtype=torch.float32)
        dx4, dxbs = nchw(dx)
        if dx4.data_ptr() != dx.data_ptr():
            raise RuntimeError("maxpool pyramid backward: gradient buffer must be per-sample dense")
        args, keep = [], []
        for lv in range(4):
            if lv < L and dys[lv] is not None:
                d4, dbs = nchw(dys[lv])
                keep.append(d4)
                args += [ptr(d4), dbs, ptr(ids[lv])]
            else:
                args += [None, 0, None]
        call("dsgan_maxpool_pyr_bwd", *args, ptr(dx4), dxbs, L, N, C, H, W, int(acc), stream())
        return (None if acc else _give(ctx.box, dx)), None


def max_pool_pyramid(x, levels):
    """[MaxPool2d(2)(x), MaxPool2d(4)(x), ..., MaxPool2d(2^levels)(x)]: one launch when the shape
    allows (H % 16 == 0, W % 64 == 0), else one max_pool2d per level."""
    N, C, H, W = x.shape
    if _lib.load().dsgan_maxpool_pyr_supported(H, W, levels):
        return list(MaxPoolPyrFn.apply(x, levels)[:levels])
    return [max_pool2d(x, 2 << lv) for lv in range(levels)]


def max_pool2d(x, k, return_indices=False):
    y, idx = MaxPoolFn.apply(x, k)
    return (y, idx) if return_indices else y


def maxpool_raw(x, k):
    """MaxPool2d(k) forward without autograd: (y, int32 plane-flat argmax)."""
    x4, xbs = nchw(x)
    N, C, H, W = x4.shape
    Ho, Wo = H // k, W // k
    y = _empty(N, C, Ho, Wo, x4)
    idx = torch.empty((N, C, Ho, Wo), device=x4.device, dtype=torch.int32)
    call("dsgan_maxpool_fwd", ptr(x4), xbs, ptr(y), C * Ho * Wo, ptr(idx), N, C, H, W, k, stream())
    return y, idx


# ------------------------------------------------------------------------------------------
# VGG16 perceptual term (DSGAN/models/vgg.py:30-42, pix2pix_model.py:180-186) as ONE autograd
# node: loss = L1(f1,r1) + L1(f2,r2) + L1(f3,r3) + L1(f0,r0), f = VGG16(fake), r = VGG16(real).
# Its backward walks the frozen VGG by hand (no weight-grads): each conv data-grad applies the
# ReLU mask of the layer below in its epilogue, and at each tapped layer one kernel forms
# (maxpool backward + L1 backward) * ReLU'  -- no standalone ReLU/L1 passes, no autograd adds.
# ------------------------------------------------------------------------------------------

def vgg_features_raw(x, blocks):
    """blocks = [(pool, [(w, b), ...]), ...] -> (feats, saved): feats = post-ReLU output of each
    block, saved = per block (pool argmax or None, input shape of the pool, [conv outputs])."""
    h = x
    feats, saved = [], []
    for pool, convs in blocks:
        idx, pin = None, None
        if pool:
            pin = tuple(h.shape)
            h, idx = maxpool_raw(h, 2)
        ys = []
        for w, b in convs:
            h = conv_fwd_raw(h, w, b, 1, 1, act="relu")
            ys.append(h)
        feats.append(h)
        saved.append((idx, pin, ys))
    return feats, saved


# ---- the same pass in channel-blocked bf16 (vggconv.hip, bf16 mode at image sizes % 256) ----
# Activations live as CB16 [N][C/16][H][W][16]: bf16 wherever the only consumers are bf16-operand
# MFMAs / ReLU signs / max (exact w.r.t. the bf16 arithmetic), fp32 for the four tapped features
# the L1 loss reads.  The backward's data-grads are stored as the bf16 the next conv consumes.

def vgg_cb16_ok(x):
    """bf16 mode and every VGG block resolution a multiple of 32 pixels wide (W % 256, H % 32)."""
    return _is16() and x.dim() == 4 and x.shape[3] % 256 == 0 and x.shape[2] % 32 == 0


def _cb16_empty(N, C, H, W, like, dtype):
    return torch.empty((N, C // 16, H, W, 16), device=like.device, dtype=dtype)


def _vgg_wt(w, dgrad):
    """bf16 weights of a VGG conv swizzled into vconv3x3's LDS image (dsgan_vconv_wtrans), cached."""
    key = (id(w), w.data_ptr(), tuple(w.shape), "vconv", dgrad, half_dtype())
    ent = _WT_CACHE.get(key)
    gen = _wgen(w)
    if ent is not None and ent[0] == gen and ent[1] == w._version and ent[2] is w:
        return ent[3]
    Co, Ci = w.shape[0], w.shape[1]
    wt = torch.empty(_lib.load().dsgan_vconv_wtrans_size(Co, Ci), device=w.device, dtype=half_dtype())
    call("dsgan_vconv_wtrans", ptr(w), ptr(wt), Co, Ci, int(dgrad), stream())
    _WT_CACHE[key] = (gen, w._version, w, wt)
    return wt


def _vconv(x, wt, bias, mask, y, N, K, M, H, W, relu, tag):
    e0 = IGEMM_TIMER.begin()
    call("dsgan_vconv3x3", ptr(x), ptr(wt), ptr(bias), ptr(mask), ptr(y), int(y.dtype == torch.float32), int(relu),
         N, K, M, H, W, stream())
    IGEMM_TIMER.end(e0, _conv_flops(N, K, M, 3, 3, H, W), (tag, N, K, H, W, M, 3, 1), "vconv_kernel",
                    _nb(x, wt, bias, mask, y))
    return y


def vgg_features_cb16(x, blocks, keep=False, real=None, outs=None, codes=None):
    """relu1_2..relu4_3 of x (NCHW fp32) as fp32 CB16 tensors; with keep, also per block (pool
    argmax or None, [bf16 CB16 outputs of the block's convs below the tapped one]) for the backward.
    real / outs: the real image's features -- every tap that is max-pooled also gets its perceptual
    L1 mean |f - real| into outs[tap] from the pool's read of f (dsgan_cb16_maxpool_l1), and with a
    `codes` dict its backward's per-element codes (sign(f - real), f > 0) in codes[tap]."""
    x, xbs = nchw(x)
    N, _, H, W = x.shape
    feats, saved = [], []
    h = None
    for bi, (pool, convs) in enumerate(blocks):
        idx = None
        if pool:
            f = feats[-1]
            C = f.shape[1] * 16
            H, W = H // 2, W // 2
            h = _cb16_empty(N, C, H, W, x, half_dtype())
            idx = torch.empty(h.shape, device=x.device, dtype=torch.uint8)
            if real is not None:
                tap = len(feats) - 1
                part = torch.empty(_lib.load().dsgan_cb16_maxpool_l1_parts(N, C, 2 * H, 2 * W), device=x.device,
                                   dtype=torch.float32)
                cd = None
                if codes is not None:
                    cd = torch.empty(f.shape, device=x.device, dtype=torch.uint8)
                    codes[tap] = cd
                call("dsgan_cb16_maxpool_l1", ptr(f), ptr(real[tap]), ptr(h), ptr(idx), ptr(cd), ptr(outs[tap:]),
                     *wsa(part), N, C, 2 * H, 2 * W, stream())
            else:
                call("dsgan_cb16_maxpool", ptr(f), ptr(h), ptr(idx), N, C, 2 * H, 2 * W, stream())
        acts = []
        for li, (w, b) in enumerate(convs):
            last = li == len(convs) - 1
            Co, Ci = w.shape[0], w.shape[1]
            y = _cb16_empty(N, Co, H, W, x, torch.float32 if last else half_dtype())
            if bi == 0 and li == 0:   # conv1_1, 3 -> 64: exact fp32 FMAs from the NCHW image
                call("dsgan_vgg_conv1_fwd", ptr(x), xbs, ptr(w), ptr(b), ptr(y), N, H, W, stream())
            else:
                _vconv(h, _vgg_wt(w, 0), b, None, y, N, Ci, Co, H, W, True, "fwd")
            if keep and not last:
                acts.append(y)
            h = y
        feats.append(h)
        saved.append((idx, acts))
    return feats, saved


def _perceptual_bwd_cb16(ctx, g):
    """Backward of PerceptualL1Fn over the CB16 pass: tap (L1 + pool backward) x ReLU', then each
    conv's data-grad x the ReLU' of the conv below in its epilogue, down to conv1_1's data-grad."""
    d, d_idx = None, None
    dx = None
    for bi in range(len(ctx.blocks) - 1, -1, -1):
        pool, convs = ctx.blocks[bi]
        idx, acts = ctx.saved[bi]
        f, r = ctx.feats[bi], ctx.real[bi]
        N, Cb, H, W, _ = r.shape
        dpre = _cb16_empty(N, Cb * 16, H, W, r, half_dtype())
        if bi in ctx.codes:
            call("dsgan_cb16_tap_bwd_codes", ptr(d), ptr(d_idx), ptr(ctx.codes[bi]), ptr(dpre), N, Cb * 16, H, W, ptr(g),
                 stream())
        else:
            call("dsgan_cb16_tap_bwd", ptr(d), ptr(d_idx), ptr(f), ptr(r), ptr(dpre), N, Cb * 16, H, W, ptr(g),
                 stream())
        for li in range(len(convs) - 1, -1, -1):
            w = convs[li][0]
            Co, Ci = w.shape[0], w.shape[1]
            if bi == 0 and li == 0:
                dx = torch.empty(ctx.fake_shape, device=r.device, dtype=torch.float32)
                call("dsgan_vgg_conv1_dgrad", ptr(dpre), ptr(w), ptr(dx), Ci * H * W, N, H, W, stream())
            else:
                out = _cb16_empty(N, Ci, H, W, r, half_dtype())
                _vconv(dpre, _vgg_wt(w, 1), None, acts[li - 1] if li > 0 else None, out, N, Co, Ci, H, W, False, "dgrad")
                dpre = out
        d, d_idx = dpre, idx
    return dx


def _sum4_raw(outs):
    """((L1(f1) + L1(f2)) + L1(f3)) + L1(f0) -- the reference's order -- in one dsgan_loss_combine
    launch (the fp32 adds of the three torch adds it replaces)."""
    import ctypes
    xp = (ctypes.c_void_p * 4)(*[outs[i:].data_ptr() for i in (1, 2, 3, 0)])
    ones, zeros = (ctypes.c_float * 4)(1, 1, 1, 1), (ctypes.c_float * 4)(0, 0, 0, 0)
    out = torch.empty((), device=outs.device, dtype=torch.float32)
    call("dsgan_loss_combine", ctypes.cast(xp, ctypes.c_void_p), ctypes.cast(ones, ctypes.c_void_p),
         ctypes.cast(zeros, ctypes.c_void_p), ctypes.cast(ones, ctypes.c_void_p), 4, 1.0, ptr(out), stream())
    return out


# the perceptual L1 of each max-pooled VGG tap from the pool's read of it (dsgan_cb16_maxpool_l1);
# DSGAN_VGG_POOL_L1=0: the separate L1 pass (A/B runs)
VGG_POOL_L1 = [os.environ.get("DSGAN_VGG_POOL_L1", "1") != "0"]


def _record_all(obj, stream):
    """record_stream(stream) on every tensor in a nest of lists / tuples / dicts."""
    if torch.is_tensor(obj):
        obj.record_stream(stream)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _record_all(o, stream)
    elif isinstance(obj, dict):
        for o in obj.values():
            _record_all(o, stream)


class PerceptualL1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fake, blocks, real_feats, side=None):
        if side is not None:
            # the forward's kernels on the side stream (the caller joins it before reading the loss);
            # the autograd node was created on the current stream, so the backward runs there, and
            # every tensor it or the caller reads is handed over to that stream
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                out = PerceptualL1Fn.forward(ctx, fake, blocks, real_feats)
            _record_all([out, ctx.saved, getattr(ctx, "feats", None), getattr(ctx, "codes", None)], main)
            return out
        ctx.box = _box(fake)
        fake, _ = nchw(fake)
        ctx.cb16 = real_feats[0].dim() == 5
        if ctx.cb16:
            # the L1 of every tap that is max-pooled comes from the pool's read of it; the others here
            outs = torch.empty(4, device=fake.device, dtype=torch.float32)
            fuse = VGG_POOL_L1[0]
            codes = {}
            feats, saved = vgg_features_cb16(fake, blocks, keep=True, real=real_feats if fuse else None, outs=outs,
                                             codes=codes)
            for i, (f, r) in enumerate(zip(feats, real_feats)):
                if i in codes:
                    continue
                call("dsgan_l1_fwd", ptr(f), ptr(r), f.numel(), ptr(outs[i:]), ptr(_loss_part(f)), stream())
            # a tap with codes needs neither its feature nor the real one in the backward
            feats = [None if i in codes else t for i, t in enumerate(feats)]
            ctx.blocks, ctx.saved, ctx.real, ctx.feats, ctx.codes = blocks, saved, real_feats, feats, codes
            ctx.fake_shape = tuple(fake.shape)
            ctx.prec = _state["prec"]
            return _sum4_raw(outs)
        feats, saved = vgg_features_raw(fake, blocks)
        outs = torch.empty(4, device=fake.device, dtype=torch.float32)
        for i, (f, r) in enumerate(zip(feats, real_feats)):
            call("dsgan_l1_fwd", ptr(f), ptr(r.contiguous()), f.numel(), ptr(outs[i:]), ptr(_loss_part(f)), stream())
        ctx.blocks, ctx.saved, ctx.real = blocks, saved, real_feats
        ctx.fake_shape = tuple(fake.shape)
        ctx.prec = _state["prec"]
        return _sum4_raw(outs)

    @staticmethod
    def backward(ctx, g):
        if ctx.cb16:
            with precision(ctx.prec):
                dx = _perceptual_bwd_cb16(ctx, g.contiguous())
            ctx.saved = ctx.real = ctx.feats = ctx.codes = None
            return _give(ctx.box, dx), None, None, None
        with precision(ctx.prec):
            g = g.contiguous()
            d, d_idx = None, None   # grad at the pool output of the block above, and that pool's argmax
            for bi in range(len(ctx.blocks) - 1, -1, -1):
                pool, convs = ctx.blocks[bi]
                idx, pin, ys = ctx.saved[bi]
                y_top = ys[-1]
                N, C, H, W = y_top.shape
                dpre = torch.empty_like(y_top)
                # tapped layer: (pool backward of the block above + L1 backward) * ReLU'
                call("dsgan_vgg_tap_bwd", ptr(d), ptr(d_idx), ptr(y_top), ptr(ctx.real[bi].contiguous()), ptr(dpre),
                     N * C, H, W, ptr(g), stream())
                for li in range(len(convs) - 1, -1, -1):
                    w = convs[li][0]
                    if li > 0:
                        # data-grad into the conv below, masked by that conv's ReLU in the epilogue
                        below = ys[li - 1]
                        dpre = conv_dgrad_raw(dpre, w, tuple(below.shape), 1, 1, gpre=below, gact="relu")
                    else:
                        in_shape = (pin[0], pin[1], pin[2] // 2, pin[3] // 2) if pool else ctx.fake_shape
                        dpre = conv_dgrad_raw(dpre, w, in_shape, 1, 1)
                d, d_idx = dpre, idx
            ctx.saved = ctx.real = None
            return _give(ctx.box, d), None, None, None


def perceptual_l1(fake, blocks, real_feats, side=None):
    """side (nullable torch.cuda.Stream): run the forward's kernels there -- the caller joins it before
    reading the loss -- while the backward stays on the current stream."""
    return PerceptualL1Fn.apply(fake, blocks, real_feats, side)


# ------------------------------------------------------------------------------------------
# MidMLKA tail (MixConvNeXtML.py:112-116):  out = GELU( IN( v * CA(v) ) + x )
# ------------------------------------------------------------------------------------------

class MidTailFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, v, x, w1, pa, w2):
        v4, vbs = nchw(v)
        N, C, H, W = v4.shape
        R = w1.shape[0]
        avg = torch.empty(N * C, device=v.device, dtype=torch.float32)
        mx = torch.empty_like(avg)
        amax = torch.empty(N * C, device=v.device, dtype=torch.int32)
        call("dsgan_plane_stats", ptr(v4), vbs, ptr(avg), ptr(mx), ptr(amax), N, C, H * W, stream())
        att = torch.empty(N * C, device=v.device, dtype=torch.float32)
        hsave = torch.empty(N * R * 2, device=v.device, dtype=torch.float32)
        call("dsgan_ca_fwd", ptr(avg), ptr(mx), ptr(w1), ptr(w2), ptr(pa), ptr(att), ptr(hsave), N, C, R, stream())
        y, mean, rstd = instnorm_raw(v4, att, x, "gelu")
        ctx.save_for_backward(v4, x, w1, pa, w2, avg, mx, amax, att, hsave, mean, rstd)
        ctx.refs = (w1, pa, w2)
        ctx.box_v, ctx.box_x = _box(v), _box(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        v, x, w1, pa, w2, avg, mx, amax, att, hsave, mean, rstd = ctx.saved_tensors
        N, C, H, W = v.shape
        R = w1.shape[0]
        dv, dx, datt = instnorm_bwd_raw(dy, v, att, x, mean, rstd, "gelu", ctx.needs_input_grad[1], True)
        davg = torch.empty(N * C, device=v.device, dtype=torch.float32)
        dmx = torch.empty_like(davg)
        w1r, par, w2r = ctx.refs
        call("dsgan_ca_bwd", ptr(datt), ptr(att), ptr(avg), ptr(mx), ptr(hsave), ptr(w1), ptr(w2), ptr(pa),
             ptr(davg), ptr(dmx), ptr(_grad_buf(w1r)), ptr(_grad_buf(w2r)), ptr(_grad_buf(par)), N, C, R,
             *wsa(torch.empty(N * (2 * R * C + 1), device=v.device, dtype=torch.float32)), stream())
        call("dsgan_plane_stats_bwd", ptr(davg), ptr(dmx), ptr(amax), ptr(dv), C * H * W, N, C, H * W, stream())
        _params_done(*ctx.refs)
        return _give(ctx.box_v, dv), _give(ctx.box_x, dx), None, None, None


def mid_tail(v, x, w1, pa, w2):
    """w1: CA.fc1 weight [C/8, C, 1, 1], pa: PReLU weight [1], w2: CA.fc2 weight [C, C/8, 1, 1]."""
    return MidTailFn.apply(v, x, w1, pa, w2)


# ------------------------------------------------------------------------------------------
# n-ary add and channel concat
# ------------------------------------------------------------------------------------------

class AddNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        ts = [nchw(t) for t in xs]
        N, C, H, W = ts[0][0].shape
        out = _empty(N, C, H, W, ts[0][0])
        import ctypes
        arr = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t, _ in ts])
        bss = (ctypes.c_long * len(ts))(*[bs for _, bs in ts])
        call("dsgan_add_n", ctypes.cast(arr, ctypes.c_void_p), ctypes.cast(bss, ctypes.c_void_p), len(ts),
             ptr(out), C * H * W, N, C * H * W, stream())
        ctx.n = len(xs)
        ctx.boxes = [_box(t) for t in xs]
        return out

    @staticmethod
    def backward(ctx, dy):
        # the same dy goes to every input: a shared input may only borrow it
        return tuple(_give(b, dy, adopt=False) for b in ctx.boxes)


def add_n(*xs):
    return AddNFn.apply(*xs)


class CatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        N, Ca, H, W = a.shape
        Cb = b.shape[1]
        out = _empty(N, Ca + Cb, H, W, a)
        copy_into(out[:, :Ca], a)
        copy_into(out[:, Ca:], b)
        ctx.Ca = Ca
        ctx.box_a, ctx.box_b = _box(a), _box(b)
        return out

    @staticmethod
    def backward(ctx, dy):
        # disjoint channel slices of dy: a shared input may adopt its slice as its buffer
        return _give(ctx.box_a, dy[:, :ctx.Ca]), _give(ctx.box_b, dy[:, ctx.Ca:])


def cat_channels(a, b):
    return CatFn.apply(a, b)


# ------------------------------------------------------------------------------------------
# Losses (0-d device tensors; backward reads the upstream grad from device memory)
# ------------------------------------------------------------------------------------------

def _loss_part(like):
    """Block-partial scratch of the deterministic loss reductions (dsgan_loss_parts floats)."""
    return torch.empty(_lib.load().dsgan_loss_parts(), device=like.device, dtype=torch.float32)


class BCELogitsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, target):
        x = x.contiguous()
        out = torch.empty((), device=x.device, dtype=torch.float32)
        call("dsgan_bce_logits_fwd", ptr(x), x.numel(), float(target), ptr(out), ptr(_loss_part(x)), stream())
        ctx.target = float(target)
        ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        dx = torch.empty_like(x)
        g = g.contiguous()
        call("dsgan_bce_logits_bwd", ptr(x), x.numel(), ctx.target, ptr(g), ptr(dx), 0, stream())
        return dx, None


def bce_with_logits(x, target):
    return BCELogitsFn.apply(x, target)


def _loss_grad(box, like, run):
    """Input-grad of a loss w.r.t. a (possibly shared, HF.share) image: a shared input whose buffer
    is owned and dense gets the grad accumulated in-kernel (run(buf, 1)); otherwise a fresh grad
    (run(d, 0)) is handed to the box or returned.  Either way the grads of a shared tensor are
    summed in arrival order, old + new, as autograd sums them."""
    buf, acc = _acc_target(box)
    if acc and buf.is_contiguous() and buf.shape == like.shape and buf.dtype == torch.float32:
        run(buf, 1)
        return None
    d = torch.empty_like(like)
    run(d, 0)
    return _give(box, d)


class L1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.box_a, ctx.box_b = _box(a), _box(b)
        a, b = a.contiguous(), b.contiguous()
        out = torch.empty((), device=a.device, dtype=torch.float32)
        call("dsgan_l1_fwd", ptr(a), ptr(b), a.numel(), ptr(out), ptr(_loss_part(a)), stream())
        ctx.save_for_backward(a, b)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        da = db = None
        if ctx.needs_input_grad[0]:
            da = _loss_grad(ctx.box_a, a, lambda d, acc: call("dsgan_l1_bwd", ptr(a), ptr(b), a.numel(), ptr(g),
                                                              ptr(d), acc, stream()))
        if ctx.needs_input_grad[1]:
            db = _loss_grad(ctx.box_b, b, lambda d, acc: call("dsgan_l1_bwd", ptr(b), ptr(a), b.numel(), ptr(g),
                                                              ptr(d), acc, stream()))
        return da, db


def l1_loss(a, b):
    return L1Fn.apply(a, b)


class TVFn(torch.autograd.Function):
    """(sum|dW| + sum|dH|) * coef over the whole batch (pix2pix_model.py:189-191, coef=1/(320*256))."""

    @staticmethod
    def forward(ctx, y, coef):
        ctx.box = _box(y)
        y = y.contiguous()
        N, C, H, W = y.shape
        out = torch.empty((), device=y.device, dtype=torch.float32)
        call("dsgan_tv_fwd", ptr(y), N * C, H, W, float(coef), ptr(out), ptr(_loss_part(y)), stream())
        ctx.coef = float(coef)
        ctx.save_for_backward(y)
        return out

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        N, C, H, W = y.shape
        g = g.contiguous()
        dy = _loss_grad(ctx.box, y, lambda d, acc: call("dsgan_tv_bwd", ptr(y), N * C, H, W, ctx.coef, ptr(g), ptr(d),
                                                        acc, stream()))
        return dy, None


def tv_loss(y, coef=1.0 / (320 * 256)):
    return TVFn.apply(y, coef)


class LossSumFn(torch.autograd.Function):
    """scale * sum_i a_i * (b_i + c_i * x_i) over 0-d fp32 losses in one launch each way
    (dsgan_loss_combine): the same fp32 roundings as the torch scalar-op chain it replaces, which
    costs one launch per multiply / add / rsub forward and per multiply backward."""

    @staticmethod
    def forward(ctx, coefs, scale, *xs):
        import ctypes
        n = len(xs)
        fa = ctypes.c_float * n
        ctx.a = fa(*[float(a) for a, _, _ in coefs])
        ctx.c = fa(*[float(c) for _, _, c in coefs])
        ctx.scale = float(scale)
        b = fa(*[float(b) for _, b, _ in coefs])
        xp = (ctypes.c_void_p * n)(*[ptr(x) for x in xs])
        out = torch.empty((), device=xs[0].device, dtype=torch.float32)
        call("dsgan_loss_combine", ctypes.cast(xp, ctypes.c_void_p), ctypes.cast(ctx.a, ctypes.c_void_p),
             ctypes.cast(b, ctypes.c_void_p), ctypes.cast(ctx.c, ctypes.c_void_p), n, ctx.scale, ptr(out), stream())
        ctx.n = n
        return out

    @staticmethod
    def backward(ctx, g):
        import ctypes
        gx = torch.empty(ctx.n, device=g.device, dtype=torch.float32)
        call("dsgan_loss_combine_bwd", ptr(g.contiguous()), ctypes.cast(ctx.a, ctypes.c_void_p),
             ctypes.cast(ctx.c, ctypes.c_void_p), ctx.n, ctx.scale, ptr(gx), stream())
        return (None, None) + tuple(gx[i] for i in range(ctx.n))


def loss_sum(terms, scale=1.0):
    """scale * (t_0 + t_1 + ...), t_i = a * (b + c * x) for terms (x, a[, b, c]) with c = +-1, summed
    left to right -- e.g. ``loss_sum([(gan, w_gan), (l1, 1), (ssim, w_ss, 1, -1)])`` is
    ``gan * w_gan + l1 + w_ss * (1 - ssim)`` rounded as torch rounds that expression.  Terms whose x
    is a python 0 (a disabled loss) are dropped, as ``0 * w + t`` is t."""
    xs, coefs = [], []
    for t in terms:
        x, a = t[0], t[1]
        b, c = (t[2], t[3]) if len(t) > 2 else (0.0, 1.0)
        if not torch.is_tensor(x):
            if x == 0 and b == 0:
                continue
            raise ValueError("loss_sum: non-tensor term %r" % (x,))
        if x.dim() != 0 or x.dtype != torch.float32 or not x.is_cuda or c not in (1, -1, 1.0, -1.0):
            raise ValueError("loss_sum: 0-d fp32 device losses and c = +-1 only")
        xs.append(x)
        coefs.append((a, b, c))
    if not xs or len(xs) > 8:
        raise ValueError("loss_sum: 1..8 tensor terms")
    return LossSumFn.apply(tuple(coefs), scale, *xs)


_WIN_CACHE = {}


def gauss_win(device, size=11, sigma=1.5):
    """_fspecial_gauss_1d (DSGAN/MS_SSIM.py:9-23), built in fp32 on the host, cached on device."""
    key = (str(device), size, sigma)
    if key not in _WIN_CACHE:
        c = torch.arange(size, dtype=torch.float) - size // 2
        g = torch.exp(-(c ** 2) / (2 * sigma ** 2))
        _WIN_CACHE[key] = (g / g.sum()).to(device)
    return _WIN_CACHE[key]


class SSIMFn(torch.autograd.Function):
    """mean SSIM of (a*real+b, a*fake+b) with data_range 1 (MS_SSIM.py:95-150); grad w.r.t. fake."""

    @staticmethod
    def forward(ctx, real, fake, a, b, data_range):
        ctx.box = _box(fake)
        real, fake = real.contiguous(), fake.contiguous()
        N, C, H, W = real.shape
        Ho, Wo = H - 10, W - 10
        coef = torch.empty((3, N * C, Ho, Wo), device=real.device, dtype=torch.float32)
        s = torch.empty((), device=real.device, dtype=torch.float32)
        win = gauss_win(real.device)
        C1 = (0.01 * data_range) ** 2
        C2 = (0.03 * data_range) ** 2
        part = torch.empty(_lib.load().dsgan_ssim_parts(N * C, H, W), device=real.device, dtype=torch.float32)
        call("dsgan_ssim_fwd", ptr(real), ptr(fake), float(a), float(b), N * C, H, W, ptr(win),
             float(C1), float(C2), ptr(coef), ptr(s), ptr(part), stream())
        cnt = float(N * C * Ho * Wo)
        ctx.save_for_backward(real, fake, coef)
        ctx.ab, ctx.cnt = (float(a), float(b)), cnt
        return s / cnt

    @staticmethod
    def backward(ctx, g):
        real, fake, coef = ctx.saved_tensors
        N, C, H, W = real.shape
        g = g.contiguous()
        dfake = _loss_grad(ctx.box, fake, lambda d, acc: call(
            "dsgan_ssim_bwd", ptr(real), ptr(fake), ctx.ab[0], ctx.ab[1], N * C, H, W, ptr(gauss_win(real.device)),
            ptr(coef), ptr(g), 1.0 / ctx.cnt, ptr(d), acc, stream()))
        return None, dfake, None, None, None


def ssim_affine(real, fake, a=0.5, b=0.5, data_range=1.0):
    return SSIMFn.apply(real, fake, a, b, data_range)


MS_SSIM_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def ms_ssim_affine(real, fake, a=1.0, b=0.0, data_range=1.0, weights=MS_SSIM_WEIGHTS, size_average=True):
    """MS-SSIM of (a*real+b, a*fake+b) (DSGAN/MS_SSIM.py:153-225), evaluation only (no autograd):
    a 0-d tensor (size_average) or the per-image values [N]."""
    import ctypes
    real, fake = real.detach().contiguous(), fake.detach().contiguous()
    if real.shape != fake.shape or real.dim() != 4:
        raise ValueError("ms_ssim: two (N,C,H,W) tensors of the same shape required")
    N, C, H, W = real.shape
    lib = _lib.load()
    work = torch.empty(lib.dsgan_ms_ssim_workspace(N, C, H, W), device=real.device, dtype=torch.float32)
    stats = torch.empty(2 * len(weights) * N * C, device=real.device, dtype=torch.float32)
    out = torch.empty(N + 1, device=real.device, dtype=torch.float32)
    wh = (ctypes.c_float * len(weights))(*[float(w) for w in weights])
    C1 = (0.01 * data_range) ** 2
    C2 = (0.03 * data_range) ** 2
    call("dsgan_ms_ssim", ptr(real), ptr(fake), float(a), float(b), N, C, H, W, ptr(gauss_win(real.device)),
         float(C1), float(C2), ctypes.cast(wh, ctypes.c_void_p), len(weights), *wsa(work), ptr(stats), ptr(out),
         stream())
    return out[N] if size_average else out[:N]


class MSSSIMFn(torch.autograd.Function):
    """Batch-mean MS-SSIM of (a*real+b, a*fake+b) (DSGAN/MS_SSIM.py:153-225, size_average=True)
    as a loss term: gradient w.r.t. fake through the 5-level pyramid (losses.hip)."""

    @staticmethod
    def forward(ctx, real, fake, a, b, data_range, weights):
        import ctypes
        real, fake = real.contiguous(), fake.contiguous()
        if real.shape != fake.shape or real.dim() != 4:
            raise ValueError("ms_ssim: two (N,C,H,W) tensors of the same shape required")
        N, C, H, W = real.shape
        L = len(weights)
        lib = _lib.load()
        work = torch.empty(lib.dsgan_ms_ssim_train_workspace(N, C, H, W, L), device=real.device, dtype=torch.float32)
        stats = torch.empty(2 * L * N * C, device=real.device, dtype=torch.float32)
        out = torch.empty(N + 1, device=real.device, dtype=torch.float32)
        wh = (ctypes.c_float * L)(*[float(w) for w in weights])
        C1, C2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
        call("dsgan_ms_ssim_fwd_train", ptr(real), ptr(fake), float(a), float(b), N, C, H, W,
             ptr(gauss_win(real.device)), float(C1), float(C2), ctypes.cast(wh, ctypes.c_void_p), L, *wsa(work),
             ptr(stats), ptr(out), stream())
        ctx.save_for_backward(real, fake, work, stats)
        ctx.args = (float(a), float(b), float(C1), float(C2), tuple(float(w) for w in weights))
        return out[N]

    @staticmethod
    def backward(ctx, g):
        import ctypes
        real, fake, work, stats = ctx.saved_tensors
        a, b, C1, C2, weights = ctx.args
        N, C, H, W = real.shape
        wh = (ctypes.c_float * len(weights))(*weights)
        dfake = torch.empty_like(fake)
        call("dsgan_ms_ssim_bwd", ptr(real), ptr(fake), a, b, N, C, H, W, ptr(gauss_win(real.device)), C1, C2,
             ctypes.cast(wh, ctypes.c_void_p), len(weights), *wsa(work), ptr(stats), ptr(g.contiguous()), ptr(dfake),
             0, stream())
        return None, dfake, None, None, None, None


def ms_ssim_loss_affine(real, fake, a=0.5, b=0.5, data_range=1.0, weights=MS_SSIM_WEIGHTS):
    """Differentiable batch-mean MS-SSIM of (a*real+b, a*fake+b); gradient w.r.t. fake only."""
    return MSSSIMFn.apply(real, fake, a, b, data_range, tuple(weights))
