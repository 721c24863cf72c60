"""Host-side plumbing of the deferred split reductions (split_reduce.hip + functional.deferred_splits),
without a GPU: the C queue's on/off flag and pending count, the Python keep-alive of scratch
tensors while a backward pass runs deferred, nesting, the off switch, and the empty flush (which
makes no HIP call)."""
import torch

from dsgan_hip import _lib
from dsgan_hip import functional as HF


def test_defer_flag_and_empty_queue():
    lib = _lib.load()
    assert lib.dsgan_split_pending() == 0
    old = lib.dsgan_split_defer(1)
    assert old == 0
    assert lib.dsgan_split_defer(0) == 1
    assert lib.dsgan_split_pending() == 0
    # an empty queue flushes without touching the device (any stream, NULL included)
    assert lib.dsgan_split_flush(None) == 0


def test_deferred_splits_keeps_scratch_alive_and_restores_state():
    lib = _lib.load()
    assert HF._DEFER_KEEP[0] is None
    t = torch.empty(8)   # (wsa only reads the pointer and size of a device tensor; a CPU one stands in)
    u = torch.empty(4)
    with HF.deferred_splits():
        assert HF._DEFER_KEEP[0] == []
        assert _lib.DEFER_HOOK[0] is not None     # _lib.call reports whether each call queued a reduction
        assert lib.dsgan_split_defer(1) == 1   # the C queue is on inside the block
        HF._keep(t)
        _lib.DEFER_HOOK[0](True)             # that call queued a reduction: its scratch is held
        assert HF._DEFER_KEEP[0][-1] is t
        HF._keep(u)
        _lib.DEFER_HOOK[0](False)            # this one queued nothing: its scratch is not held
        assert all(x is not u for x in HF._DEFER_KEEP[0]) and not HF._DEFER_CAND
        with HF.deferred_splits():          # nested: a no-op, the outer block owns the flush
            assert HF._DEFER_KEEP[0] and HF._DEFER_KEEP[0][-1] is t
    assert HF._DEFER_KEEP[0] is None and _lib.DEFER_HOOK[0] is None
    assert lib.dsgan_split_defer(0) == 0       # turned off again at the block's end
    assert lib.dsgan_split_pending() == 0


def test_deferred_splits_off_switch_and_exception_path():
    lib = _lib.load()
    HF.DEFER_SPLITS[0] = False
    try:
        with HF.deferred_splits():
            assert HF._DEFER_KEEP[0] is None
            assert lib.dsgan_split_defer(0) == 0   # never turned on
    finally:
        HF.DEFER_SPLITS[0] = True
    try:
        with HF.deferred_splits():
            raise ValueError("backward failed")
    except ValueError:
        pass
    assert HF._DEFER_KEEP[0] is None
    assert lib.dsgan_split_defer(0) == 0


def test_keep_outside_deferral_is_a_passthrough():
    t = torch.empty(3)
    assert HF._keep(t) is t
    assert HF._DEFER_KEEP[0] is None
