# touched-op tests (VGG conv1, CA plane stats, MidMLKA tail, step determinism), rocprofv3 kernel stats -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_vgg_cb16_gpu.py tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_pwf32_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "conv or plane_stats or mid_tail or bitwise or refresh or step or disc" > gpurun_out/r3l_tests.log 2>&1 || { tail -30 gpurun_out/r3l_tests.log; exit 1; }
tail -2 gpurun_out/r3l_tests.log
bash tools/gpu_prof.sh || exit 1
grep -iE "channel_sum|wconv" gpurun_out/prof_top.txt | cut -c1-160
tail -1 gpurun_out/prof_top.txt
