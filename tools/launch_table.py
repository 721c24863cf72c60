"""Per-launch table of the timed contraction launches of one bench step (HIP events):
family, tag (mode, N, Cin, H, W, Cout, KH, stride), ms, TFLOP/s, algorithmic GB/s.
usage: python tools/launch_table.py [--family pwgemm_kernel] [--batch 16] [--size 256]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default=None)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    a = ap.parse_args()
    from dsgan_hip import functional as HF
    from options.train_options import default_train_opt
    from models import create_model
    from oracle.recipe import synth_pair
    torch.manual_seed(20)
    m = create_model(default_train_opt(gpu_ids=[0], precision="bf16", batchSize=a.batch, cuda_graph=0))
    A, B = synth_pair(a.batch, a.size, seed=0)
    m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * a.batch, "B_paths": [""] * a.batch})
    for _ in range(3):
        m.optimize_parameters()
    torch.cuda.synchronize()
    HF.IGEMM_TIMER.rec, HF.AUX_TIMER.rec = [], []
    HF.IGEMM_TIMER.on = HF.AUX_TIMER.on = True
    m.optimize_parameters()
    torch.cuda.synchronize()
    HF.IGEMM_TIMER.on = HF.AUX_TIMER.on = False
    rows = []
    for r in HF.IGEMM_TIMER.rec + HF.AUX_TIMER.rec:
        ms = r[0].elapsed_time(r[1])
        if a.family and r[4] != a.family:
            continue
        rows.append((ms, r[4], r[3], r[2], r[5]))
    rows.sort(key=lambda t: -t[0])
    tot = sum(t[0] for t in rows)
    print("%d launches, %.3f ms" % (len(rows), tot))
    fam = {}
    for ms, f, _, fl, by in rows:
        e = fam.setdefault(f, [0, 0.0, 0.0, 0.0])
        e[0] += 1; e[1] += ms; e[2] += fl; e[3] += by
    for f, (n, ms, fl, by) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print("  %-20s %4d launches %8.3f ms %7.1f TF/s %7.1f GB/s" % (f, n, ms, fl / ms / 1e9, by / ms / 1e6))
    for ms, fam, tag, fl, by in rows:
        print("%8.1f us  %-18s %-42s %7.1f TF/s %7.1f GB/s %8.1f MB" % (ms * 1e3, fam, str(tag), fl / ms / 1e9,
                                                                        by / ms / 1e6, by / 1e6))


if __name__ == "__main__":
    main()
