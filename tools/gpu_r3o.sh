# adam paths + model/step tests, then kernel stats -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "adam or bitwise or step or fp16 or pool or vgg or loss or model or ddp" > gpurun_out/r3o_tests.log 2>&1 || { tail -30 gpurun_out/r3o_tests.log; exit 1; }
tail -2 gpurun_out/r3o_tests.log
bash tools/gpu_prof.sh || exit 1
grep -ciE "FillFunctor<int>" gpurun_out/prof_stats.csv || true
grep -i adam gpurun_out/prof_stats.csv | cut -c1-200
tail -1 gpurun_out/prof_top.txt
