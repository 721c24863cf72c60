set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/wconv_micro.py 2>&1 | grep -v amdgpu.ids > gpurun_out/wc.log || exit 1
cat gpurun_out/wc.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wconv or conv2d or conv_transpose or model_gpu or configs" > gpurun_out/tt.log 2>&1; rc=$?
tail -2 gpurun_out/tt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-160; exit $rc
