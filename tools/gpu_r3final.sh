# round-3 final pass on the current tree: full -m gpu suite, smoke(), default bench line (quality +
# cpu_baseline legs), rocprofv3 kernel stats, PMC HBM traffic, MFMA/LDS counters, per-launch table
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.txt 2>&1 || { tail -40 gpurun_out/gpu_tests_final.txt; exit 1; }
tail -2 gpurun_out/gpu_tests_final.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.txt 2>&1 || { tail -20 gpurun_out/smoke_final.txt; exit 1; }
tail -1 gpurun_out/smoke_final.txt
timeout -k 10 800 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-300
bash tools/gpu_profiles.sh || exit 1
head -24 gpurun_out/launches_all.txt | tail -19
