# Development GPU pass: all parity tests, one bench line (no CPU legs), the per-launch GEMM breakdown.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -15 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/igemm_breakdown.py bf16 > gpurun_out/brk.log 2>&1
