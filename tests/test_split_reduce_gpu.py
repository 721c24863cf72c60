"""split_reduce.hip: the fixed-order split reduction every weight-grad finishes with, immediate and
deferred (queued, then flushed as batched multi-segment launches), against a numpy float32
restatement of its order of additions (bit-exact), and the deferred training step against the
immediate one (bitwise-equal gradients, parameters and losses)."""
import random

import numpy as np
import pytest
import torch


pytestmark = pytest.mark.gpu


def canon_sum(ws):
    """sum over rows of ws [S, MN] in split_reduce.hip's order (float32 adds, exact emulation)."""
    S, MN = ws.shape
    f32 = np.float32
    if S > 64 and MN < 65536:   # group rows: ((p0 + p1) + p2) + p3 over 16 splits each
        rows = []
        for g in range((S + 15) // 16):
            s0, s1 = 16 * g, min(S, 16 * g + 16)
            q = [np.zeros(MN, f32) for _ in range(4)]
            for s in range(s0, s1):
                q[(s - s0) & 3] = q[(s - s0) & 3] + ws[s]
            rows.append(((q[0] + q[1]) + q[2]) + q[3])
    else:
        rows = list(ws)
    J = 4 if len(rows) <= 8 else 16
    t = np.zeros(MN, f32)
    for lane in range(J):
        a = np.zeros(MN, f32)
        for r in range(lane, len(rows), J):
            a = a + rows[r]
        t = t + a
    return t


def _lib():
    import dsgan_hip
    from dsgan_hip import _lib as L
    dsgan_hip.require_gpu()
    return L


@pytest.mark.parametrize("S,MN,off", [
    (1, 7, 0), (3, 64, 0), (8, 4096, 0), (9, 4096, 1), (16, 1000, 0), (64, 8192, 0),
    (65, 8192, 0), (100, 513, 1), (640, 8192, 0), (200, 70000, 0), (300, 1, 0), (77, 12, 3),
])
def test_split_reduce_order_bit_exact(S, MN, off):
    """Immediate form (dsgan_colsum -> launch_split_reduce): float4 and scalar element forms (off
    misaligns the rows), 4 / 16 lanes, with and without the 16-split group rows."""
    L = _lib()
    rng = np.random.default_rng(S * 1000 + MN)
    ws = rng.standard_normal((S, MN)).astype(np.float32) * np.float32(3.0)
    out0 = rng.standard_normal(MN).astype(np.float32)
    dev = torch.empty(S * MN + off, device="cuda")
    dev[off:] = torch.from_numpy(ws.reshape(-1)).cuda()
    out = torch.from_numpy(out0).cuda()
    L.call("dsgan_colsum", L.ptr(dev) + 4 * off, S, MN, L.ptr(out), L.stream())
    torch.cuda.synchronize()
    exp = out0 + canon_sum(ws)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), exp.view(np.uint32))


def test_deferred_queue_overlap_and_order():
    """Deferred mode: reductions queued across calls (same output twice, disjoint outputs, > RS_MAX
    segments) and flushed in batched launches give the immediate form's bits, in queue order."""
    L = _lib()
    lib = L.load()
    rng = np.random.default_rng(5)
    cases = [(9, 4096), (65, 8192), (3, 100), (17, 64)] * 6 + [(640, 8192)]
    parts, outs = [], []
    for i, (S, MN) in enumerate(cases):
        parts.append(rng.standard_normal((S, MN)).astype(np.float32))
    shared = np.zeros(4096, np.float32)   # cases 0, 4, 8, ... (S = 9) all add into one output
    dev_parts = [torch.from_numpy(p.reshape(-1)).cuda() for p in parts]
    dev_shared = torch.from_numpy(shared).cuda()
    dev_outs = []
    assert lib.dsgan_split_pending() == 0
    old = lib.dsgan_split_defer(1)
    try:
        for i, (S, MN) in enumerate(cases):
            if MN == 4096:
                tgt = dev_shared
            else:
                tgt = torch.zeros(MN, device="cuda")
                dev_outs.append((i, tgt))
            L.call("dsgan_colsum", L.ptr(dev_parts[i]), S, MN, L.ptr(tgt), L.stream())
        assert lib.dsgan_split_pending() == len(cases)
        assert float(dev_shared.abs().sum()) == 0.0   # nothing ran yet
    finally:
        lib.dsgan_split_defer(old)
    L.call("dsgan_split_flush", L.stream())
    assert lib.dsgan_split_pending() == 0
    torch.cuda.synchronize()
    exp_shared = np.zeros(4096, np.float32)
    for i, (S, MN) in enumerate(cases):
        if MN == 4096:
            exp_shared = exp_shared + canon_sum(parts[i])
    assert np.array_equal(dev_shared.cpu().numpy().view(np.uint32), exp_shared.view(np.uint32))
    for i, t in dev_outs:
        assert np.array_equal(t.cpu().numpy().view(np.uint32), canon_sum(parts[i]).view(np.uint32)), i


def test_flush_from_a_foreign_stream_orders_it():
    """a flush called with another stream than the queued reductions' launches them on
    their own stream and makes the caller's stream wait for them (an event): the queue is empty
    afterwards and work on the caller's stream reads the reduced values."""
    L = _lib()
    lib = L.load()
    part = torch.randn(9, 64, device="cuda")
    out = torch.zeros(64, device="cuda")
    old = lib.dsgan_split_defer(1)
    try:
        L.call("dsgan_colsum", L.ptr(part), 9, 64, L.ptr(out), L.stream())
    finally:
        lib.dsgan_split_defer(old)
    assert lib.dsgan_split_pending() == 1
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    L.call("dsgan_split_flush", side.cuda_stream)
    assert lib.dsgan_split_pending() == 0
    with torch.cuda.stream(side):
        copy = out.clone()          # ordered after the reduction by the flush's event
    torch.cuda.synchronize()
    assert torch.equal(copy.cpu(), torch.from_numpy(canon_sum(part.cpu().numpy())))


@pytest.mark.parametrize("prec,size", [("bf16", 256), ("fp32", 64), ("fp16", 128)])
def test_step_deferred_equals_immediate(prec, size):
    """One G+D training step with the backward passes' split reductions deferred (the default) and
    immediate: bitwise-equal flat gradients, updated parameters and losses (every parameter gets one
    weight-grad per backward, so batching the reductions changes no order of additions)."""
    import dsgan_hip
    from dsgan_hip import functional as HF
    from options.train_options import default_train_opt
    from models import create_model
    from oracle import dsgan_cpu as O
    from oracle.recipe import make_params, synth_pair
    dsgan_hip.require_gpu()
    outs = []
    for defer in (True, False):
        HF.DEFER_SPLITS[0] = defer
        try:
            random.seed(20)
            torch.manual_seed(20)
            m = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision=prec))
            for net, pr in ((m.netG, make_params(O.g_param_spec(), "ref", 1000)),
                            (m.netD, make_params(O.d_param_spec(), "ref", 5000)),
                            (m.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
                with torch.no_grad():
                    for k, v in net.state_dict().items():
                        v.copy_(pr[k])
            A, B = synth_pair(2, size, seed=8)
            m.set_input({"A": A, "B": B, "A_paths": ["a"] * 2, "B_paths": ["b"] * 2})
            m.optimize_parameters()
            torch.cuda.synchronize()
            assert dsgan_hip._lib.load().dsgan_split_pending() == 0
            outs.append((m.flatG.grad.clone(), m.flatD.grad.clone(), m.flatG.data.clone(), m.flatD.data.clone(),
                         torch.stack([m.loss_G.detach(), m.loss_D.detach(), m.loss_ssim.detach()])))
            del m
        finally:
            HF.DEFER_SPLITS[0] = True
    for a, b in zip(*outs):
        assert torch.equal(a, b)
