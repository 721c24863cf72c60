# GPU check used during development: parity tests, then one bench line and the GEMM breakdown.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1; rc=$?; tail -15 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1 &&
timeout -k 10 300 python tools/igemm_breakdown.py bf16 > gpurun_out/brk.log 2>&1
