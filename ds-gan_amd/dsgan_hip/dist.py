"""Data-parallel gradient exchange: one process per GPU, torch.distributed over RCCL ("nccl"
backend on ROCm), replacing the reference's single-process nn.DataParallel
(DSGAN/models/networks.py:74-77).

Per step there are exactly two exchanges, both on flat fp32 gradient buffers:
  1. D grads (0.70 M params, 2.8 MB) after backward_D -- must land before optimizer_D.step(),
     because the G step reads the updated D;
  2. G grads (22.4 M params, 89.7 MB) after backward_G, in ``bucket_mb`` chunks so several
     RCCL rings can stream over the 7 xGMI links.
Averaging = SUM then a HIP scale by 1/world (gloo, used by the CPU tests, has no AVG op).
"""
import torch
import torch.distributed as dist

from ._lib import call, ptr, stream


def world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def broadcast_params(flat, src=0):
    if world_size() > 1:
        dist.broadcast(flat.data, src)


def _scale(t, a):
    if t.is_cuda:
        call("dsgan_scale", ptr(t), float(a), t.numel(), stream())
    else:  # gloo CPU rehearsal of the exchange (tests only; no compute path runs on CPU)
        t.mul_(a)


def allreduce_mean_(buf, bucket_mb=32):
    """In-place mean of a flat fp32 buffer over all ranks."""
    W = world_size()
    if W == 1:
        return buf
    n = buf.numel()
    step = max(1, int(bucket_mb * (1 << 20) // 4))
    works = [dist.all_reduce(buf[o:o + step], op=dist.ReduceOp.SUM, async_op=True) for o in range(0, n, step)]
    for w in works:
        w.wait()
    _scale(buf, 1.0 / W)
    return buf
