"""Captured RCCL all-reduces back to back vs interleaved with compute (1-rank "nccl" group).

Round-6 bisection of tests/test_ddp_gpu.py::test_one_rank_rccl_exchange_is_bitwise_neutral: the
G-bucket all-reduces launched in strict index order (some from a later hook than the one that
completed them, several per hook) replayed wrong values from the HIP graph; launched at completion
they did not (that order also issues several per hook, so the burst alone is not it).  This tool
captures K async in-place AVG all-reduces of disjoint slices of one buffer -- a 1-rank AVG is the
identity -- issued (a) back to back, (b) with a small kernel on the capture stream between them,
from the capturing thread or from a second thread (the autograd engine's), replays the graph a few
times and reports whether the buffer kept its values.  Prints one line per arm.
"""
import os
import sys
import threading

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29631")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    n, k = 1 << 22, 6
    buf = torch.empty(n, device="cuda")
    side = torch.zeros(1 << 16, device="cuda")
    cuts = [i * n // k for i in range(k + 1)]
    ok_all = True
    for burst in (True, False):
        for threaded in (False, True):
            # eager warm-up collective (the step before the capture runs eager)
            dist.all_reduce(buf[:1024], op=dist.ReduceOp.AVG)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            works = []

            def issue():
                cs = torch.cuda.current_stream()
                for i in range(k):
                    if not burst:
                        side.add_(1.0)
                    works.append(dist.all_reduce(buf[cuts[i]:cuts[i + 1]], op=dist.ReduceOp.AVG, async_op=True))
                return cs

            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                side.add_(1.0)
                if threaded:
                    cap = torch.cuda.current_stream()

                    def run():
                        with torch.cuda.stream(cap):
                            issue()
                    t = threading.Thread(target=run)
                    t.start()
                    t.join()
                else:
                    issue()
                for w in works:
                    w.wait()
                side.add_(1.0)
            bad = 0
            for rep in range(5):
                ref = torch.randn(n, device="cuda", generator=torch.Generator("cuda").manual_seed(rep))
                buf.copy_(ref)
                g.replay()
                torch.cuda.synchronize()
                bad += int((buf != ref).sum().item())
            ok_all &= bad == 0
            print("arm burst=%d threaded=%d: %d wrong elements over 5 replays" % (burst, threaded, bad), flush=True)
            del g
    dist.destroy_process_group()
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
