# full -m gpu suite, C2 bench line, per-launch table, rocprofv3 kernel stats, PMC passes -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_i.txt 2>&1 || { tail -40 gpurun_out/gpu_tests_i.txt; exit 1; }
tail -3 gpurun_out/gpu_tests_i.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quality > gpurun_out/bench_i.log 2>&1 || { tail -20 gpurun_out/bench_i.log; exit 1; }
tail -1 gpurun_out/bench_i.log | cut -c1-400
timeout -k 10 200 python tools/launch_table.py > gpurun_out/launches_i.txt 2>&1 || exit 1
head -24 gpurun_out/launches_i.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_i -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality > gpurun_out/prof_i.log 2>&1 || { tail -20 gpurun_out/prof_i.log; exit 1; }
find gpurun_out/prof_i -name "*kernel_stats.csv" -exec cp {} gpurun_out/rocprof_stats_i.csv \;
rm -rf gpurun_out/prof_i
bash tools/gpu_pmc.sh || exit 1
rm -rf gpurun_out/pmcf gpurun_out/pmcw
bash tools/gpu_mfma_pmc.sh || exit 1
