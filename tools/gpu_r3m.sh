# full -m gpu suite, rocprofv3 kernel stats of the bench -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_m.txt 2>&1 || { tail -40 gpurun_out/gpu_tests_m.txt; exit 1; }
tail -2 gpurun_out/gpu_tests_m.txt
bash tools/gpu_prof.sh || exit 1
grep -iE "split_reduce" gpurun_out/prof_top.txt | cut -c1-160
tail -1 gpurun_out/prof_top.txt
