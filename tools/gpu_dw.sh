# dwconv check: parity tests, kernel timings at the DS-GAN shapes (tiles-per-workgroup 4 vs 1), one bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dwconv or full_step" > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/dw_micro.py > gpurun_out/dw.log 2>&1; rc=$?; cat gpurun_out/dw.log | grep N=; [ $rc -eq 0 ] || exit $rc
DSGAN_DW_TPW=1 timeout -k 10 120 python tools/dw_micro.py > gpurun_out/dw1.log 2>&1; rc=$?; cat gpurun_out/dw1.log | grep N=; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-250; exit $rc
