# touched-op tests, pw knob A/B (gp prefetch, epilogue-heavy tile choices), step launch table -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_vgg_cb16_gpu.py tests/test_ops_gpu.py tests/test_pwf32_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv1 or pw or vgg or refresh" > gpurun_out/r3j_tests.log 2>&1 || { tail -30 gpurun_out/r3j_tests.log; exit 1; }
tail -2 gpurun_out/r3j_tests.log
timeout -k 10 400 python -u tools/pw_bench.py --only gp --arm "" --arm "8=0" --arm "7=1" --arm "7=3" --arm "6=1" --arm "6=2" > gpurun_out/r3j_pwbench.log 2>&1 || { tail -30 gpurun_out/r3j_pwbench.log; exit 1; }
cat gpurun_out/r3j_pwbench.log
timeout -k 10 200 python tools/launch_table.py > gpurun_out/launches_j.txt 2>&1 || exit 1
head -24 gpurun_out/launches_j.txt | tail -19
grep -E "vgg_conv1|conv1" gpurun_out/launches_j.txt | head
