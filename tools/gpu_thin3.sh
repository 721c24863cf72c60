set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "model_gpu or configs or conv2d or pconv or perceptual or tap_conv or determin" > gpurun_out/tt.log 2>&1; rc=$?
tail -3 gpurun_out/tt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/launch_table.py > gpurun_out/launches.txt 2>&1; rc=$?; grep -E "pconv_kernel" gpurun_out/launches.txt | head; exit $rc
