"""Which gradient sums does one training step issue as separate add_n launches?  Wraps
functional._add_n_raw to log the shape of every sum (the grads of a shared tensor that no consumer
could accumulate in-kernel), runs eager steps of the bench model and prints a table.

    python tools/addn_trace.py [--steps 2]
"""
import argparse
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    import dsgan_hip
    from dsgan_hip import functional as HF
    from options.train_options import default_train_opt
    from models import create_model
    from oracle.recipe import synth_pair
    dsgan_hip.require_gpu()
    torch.manual_seed(20)
    model = create_model(default_train_opt(gpu_ids=[0], precision="bf16", batchSize=16, cuda_graph=0))
    A, B = synth_pair(16, 256, seed=0)
    A, B = A.cuda(), B.cuda()
    log = collections.Counter()
    orig = HF._add_n_raw

    def wrapped(out, ts):
        where = [f for f in traceback.extract_stack(limit=8)[:-1] if "functional.py" in f.filename]
        caller = "%s:%d" % (os.path.basename(where[-1].filename), where[-1].lineno) if where else "?"
        log[(tuple(out.shape), len(ts), caller)] += 1
        return orig(out, ts)

    HF._add_n_raw = wrapped
    for _ in range(a.steps):
        model.set_input({"A": A, "B": B, "A_paths": [""] * 16, "B_paths": [""] * 16})
        model.optimize_parameters()
    torch.cuda.synchronize()
    tot = 0
    for (shape, n, caller), c in sorted(log.items(), key=lambda kv: -kv[1] * int(torch.tensor(kv[0][0]).prod())):
        mb = 4 * (n + 1) * int(torch.tensor(shape).prod()) / 1e6
        tot += mb * c
        print("%-28s terms=%d  x%-3d  %8.1f MB each  (%s)" % (shape, n, c // a.steps, mb, caller))
    print("total %.1f MB per step" % (tot / a.steps))


if __name__ == "__main__":
    main()
