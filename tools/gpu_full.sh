# Full GPU pass: parity tests, bench line (with CPU baseline), rocprofv3 kernel stats of the bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -8 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality > gpurun_out/prof.log 2>&1 && tail -1 gpurun_out/prof.log
