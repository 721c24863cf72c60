# the -m gpu suite, the C2 bench line, the per-launch table (HIP events) -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests_new.sh "$@" || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quality > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | cut -c1-300
timeout -k 10 200 python tools/launch_table.py > gpurun_out/launches_all.txt 2>&1 || exit $?
head -22 gpurun_out/launches_all.txt
