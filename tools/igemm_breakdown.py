"""Per-launch implicit-GEMM timing over one bench step (HIP events), aggregated by shape."""
import os, sys, collections
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
from dsgan_hip import functional as HF
from options.train_options import default_train_opt
from models import create_model
from oracle.recipe import synth_pair

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
opt = default_train_opt(gpu_ids=[0], precision=prec, cuda_graph=0)
m = create_model(opt)
A, Bi = synth_pair(B, 256, 0)
m.set_input({"A": A.cuda(), "B": Bi.cuda(), "A_paths": [""] * B, "B_paths": [""] * B})
for _ in range(2):
    m.optimize_parameters()
torch.cuda.synchronize()
HF.IGEMM_TIMER.on = True
m.optimize_parameters()
HF.IGEMM_TIMER.on = False
rows = HF.IGEMM_TIMER.table()
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
fams = HF.IGEMM_TIMER.families()
for ms, fl, tag in rows:
    a = agg[tag]; a[0] += 1; a[1] += ms; a[2] += fl
tot = sum(a[1] for a in agg.values())
print("total igemm ms %.2f over %d launches" % (tot, len(rows)))
print("%-8s %3s %5s %4s %4s %5s %2s %2s | %4s %8s %7s %7s  %s" % ("mode", "N", "Cin", "H", "W", "Cout", "K", "s", "cnt", "ms", "TF/s", "GB/s*", "kernel"))
for tag, (c, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:80]:
    mode, N, Cin, H, W, Cout, K, s, fam = tag
    Ho = (H + 2 * (K // 2 if K != 4 else 1) - K) // s + 1
    # fp32 bytes of the three operands at minimum
    if mode == "fwd":
        by = 4 * (N * Cin * H * W + N * Cout * Ho * Ho + Cout * Cin * K * K)
    elif mode == "dgrad":
        by = 4 * (N * Cin * H * W + N * Cout * Ho * Ho + Cout * Cin * K * K)
    else:
        by = 4 * (N * Cin * H * W + N * Cout * Ho * Ho)
    print("%-8s %3d %5d %4d %4d %5d %2d %2d | %4d %8.3f %7.1f %7.0f  %s" % (mode, N, Cin, H, W, Cout, K, s, c, ms, fl / (ms * 1e-3) / 1e12, by * c / (ms * 1e-3) / 1e9, fam))
