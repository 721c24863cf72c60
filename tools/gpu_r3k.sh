# MLP tests, step launch table, rocprofv3 kernel stats of the bench -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mlp or block or bitwise or refresh" > gpurun_out/r3k_tests.log 2>&1 || { tail -30 gpurun_out/r3k_tests.log; exit 1; }
tail -2 gpurun_out/r3k_tests.log
timeout -k 10 200 python tools/launch_table.py > gpurun_out/launches_k.txt 2>&1 || exit 1
head -24 gpurun_out/launches_k.txt | tail -19
grep mlp_ gpurun_out/launches_k.txt | head -12
bash tools/gpu_prof.sh || exit 1
head -45 gpurun_out/prof_top.txt
