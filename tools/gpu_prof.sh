# rocprofv3 kernel stats of a short bench run (no CPU legs), summarised on the box -> gpurun_out/prof_stats.csv
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality --no-train-equiv > gpurun_out/prof.log 2>&1; rc=$?
tail -1 gpurun_out/prof.log | cut -c1-300
# 15 executed steps: bench.py with HIP graphs runs 1 eager warm step, 2 warmup replays, 10 timed replays and
# 2 eager steps that time the roofline leg (bench.EAGER_TIMING_STEPS)
python3 tools/prof_stats.py gpurun_out/prof/run_results.db gpurun_out/prof_stats.csv --steps 15 > gpurun_out/prof_top.txt 2>&1
python3 tools/prof_dispatch.py gpurun_out/prof/run_results.db gpurun_out/prof_dispatch.csv --last 786 || true
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/prof_kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/prof
exit $rc
