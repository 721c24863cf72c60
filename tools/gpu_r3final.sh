# round-3 final artifacts of the current tree: default bench line (quality + cpu_baseline legs), rocprofv3 kernel
# stats, PMC HBM traffic, MFMA/LDS counters, per-launch table -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 800 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-300
bash tools/gpu_profiles.sh || exit 1
head -24 gpurun_out/launches_all.txt | tail -19
