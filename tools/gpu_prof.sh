# rocprofv3 kernel stats of a short bench run (no CPU legs) -> gpurun_out/prof/run_results.db
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality > gpurun_out/prof.log 2>&1; rc=$?; tail -1 gpurun_out/prof.log | cut -c1-300; exit $rc
