set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "pw_mlp or conv2d" > gpurun_out/t7.log 2>&1; rc=$?; tail -3 gpurun_out/t7.log; [ $rc -eq 0 ] || exit $rc
DSGAN_PW_BM256=0 timeout -k 10 200 python tools/igemm_breakdown.py > gpurun_out/ib_off.log 2>&1 &&
timeout -k 10 200 python tools/igemm_breakdown.py > gpurun_out/ib_on.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality > gpurun_out/bench7.log 2>&1; rc=$?; tail -1 gpurun_out/bench7.log | cut -c1-250; exit $rc
