"""Data-parallel gradient exchange: one process per GPU, torch.distributed over RCCL ("nccl"
backend on ROCm), replacing the reference's single-process nn.DataParallel
(DSGAN/models/networks.py:74-77).

Per step there are exactly two exchanges, both on flat fp32 gradient buffers (dsgan_hip.flat):
  1. D grads (0.70 M params, 2.8 MB) after backward_D, one all-reduce that must land before
     optimizer_D.step(): the G step reads the updated D (DSGAN/models/pix2pix_model.py:204-217);
  2. G grads (22.4 M params, 89.7 MB) in buckets that start DURING backward_G (``GradBuckets``):
     the G flat buffer is laid out in backward order, every autograd Function reports the
     parameters whose weight-grads it has launched (functional.GRAD_READY), and a bucket whose
     parameters are all reported is all-reduced on RCCL's stream while the rest of the backward
     keeps the CUs busy.  optimizer_G.step() waits for the buckets.
Averaging: ReduceOp.AVG on RCCL; SUM then 1/world on gloo (the CPU rehearsal used by the
tests has no AVG).
"""
import torch
import torch.distributed as dist

from ._lib import call, ptr, stream
from . import functional as HF


def world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def backend():
    """The process group's backend ("nccl" = RCCL on ROCm, "gloo"), or None without one."""
    return dist.get_backend() if dist.is_available() and dist.is_initialized() else None


def all_ranks_true(flag, device):
    """True when ``flag`` holds on every rank (one tiny MIN all-reduce; the flag itself on one rank).
    The graph step uses it so that every rank replays captured graphs, or none does."""
    if world_size() == 1:
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device if backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def broadcast_params(flat, src=0):
    if world_size() > 1:
        dist.broadcast(flat.data, src)


def _scale(t, a):
    if t.is_cuda:
        call("dsgan_scale", ptr(t), float(a), t.numel(), stream())
    else:  # gloo CPU rehearsal of the exchange (tests only; no compute path runs on CPU)
        t.mul_(a)


def _avg_op():
    return dist.ReduceOp.AVG if dist.get_backend() == "nccl" else None


def _allreduce_avg(t, async_op):
    op = _avg_op()
    return dist.all_reduce(t, op=op if op is not None else dist.ReduceOp.SUM, async_op=async_op)


def _post_scale(buf, W):
    if _avg_op() is None:
        _scale(buf, 1.0 / W)


def allreduce_mean_(buf, bucket_mb=32, force=False):
    """In-place mean of a flat fp32 buffer over all ranks (blocking for the caller's stream).
    One rank skips the collective unless ``force`` (the 1-rank RCCL test exercises it)."""
    W = world_size()
    if W == 1 and not force:
        return buf
    n = buf.numel()
    step = max(1, int(bucket_mb * (1 << 20) // 4))
    works = [_allreduce_avg(buf[o:o + step], True) for o in range(0, n, step)]
    for w in works:
        w.wait()
    _post_scale(buf, W)
    return buf


class GradBuckets:
    """Bucketed all-reduce of one flat gradient buffer, overlapped with the backward that fills it.

    ``layout`` = [(param, offset, numel)] in buffer order.  Buckets are contiguous ranges of about
    ``bucket_mb`` cut at parameter boundaries; ``arm()`` before the backward, ``ready(params)``
    from functional.GRAD_READY as weight-grads are launched, ``finish()`` after the backward:
    launches the buckets that are not complete (parameters never reported) and waits for all of them.

    A bucket starts when its last parameter is reported.  Collectives pair up across ranks by issue
    order, so the launch sequence is the order in which the backward completes the buckets: the
    autograd engine runs the same graph's nodes in the same order on every rank, so every rank
    issues the same sequence (tests/test_host_cpu.py::test_grad_buckets_sequence_follows_completion).
    Round 6 tried a strict index-order rule (bucket i waits for every bucket before it, whatever the
    report order): it launched some buckets from a later hook than the one that completed them, and
    the step captured that way replayed wrong gradients (bisected to the rule on
    tests/test_ddp_gpu.py::test_one_rank_rccl_exchange_is_bitwise_neutral; a capture of plain
    back-to-back all-reduces, tools/rccl_graph_burst.py, does not show it) -- not kept."""

    def __init__(self, grad, layout, bucket_mb=24):
        self.grad = grad
        self.buckets = []          # [start, end, set(param ids)]
        self.owner = {}            # param id -> bucket index
        lim = int(bucket_mb * (1 << 20) // 4)
        cur = None
        for p, off, n in layout:
            if cur is None or (off + n - cur[0] > lim and cur[2]):
                if cur is not None:
                    cur[1] = off
                cur = [off, off + n, set()]
                self.buckets.append(cur)
            cur[2].add(id(p))
            cur[1] = off + n
            self.owner[id(p)] = len(self.buckets) - 1
        self.buckets[-1][1] = grad.numel()
        self.pending = None
        self.works = None
        self.launched = None
        self.sequence = []         # bucket indices in launch order (this step)

    def arm(self):
        self.pending = [set(b[2]) for b in self.buckets]
        self.works = []
        self.launched = [False] * len(self.buckets)
        self.sequence = []
        HF.GRAD_READY[0] = self.ready

    def _launch(self, i):
        if not self.launched[i]:
            HF.split_flush()   # the bucket's weight-grads may still sit in the deferred split reductions
            s, e = self.buckets[i][0], self.buckets[i][1]
            self.launched[i] = True
            self.sequence.append(i)
            self.works.append(_allreduce_avg(self.grad[s:e], True))

    def ready(self, params):
        for p in params:
            i = self.owner.get(id(p))
            if i is None or self.launched[i]:
                continue
            self.pending[i].discard(id(p))
            if not self.pending[i]:
                self._launch(i)

    def finish(self):
        HF.GRAD_READY[0] = None
        for i in range(len(self.buckets)):
            self._launch(i)
        for w in self.works:
            w.wait()
        _post_scale(self.grad, world_size())
        n_early = sum(1 for i in range(len(self.buckets)) if not self.pending[i])
        self.pending = self.works = None
        return n_early
