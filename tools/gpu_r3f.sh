# selected -m gpu tests ($1: -k expression), a micro-benchmark ($2: tools/ script), the C2 bench
# line and the per-launch table -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests_new.sh tests -k "$1" || exit $?
if [ -n "$2" ]; then timeout -k 10 200 python $2 > gpurun_out/micro.log 2>&1 || exit $?; cat gpurun_out/micro.log; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quality > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | cut -c1-300
timeout -k 10 200 python tools/launch_table.py > gpurun_out/launches_all.txt 2>&1 || exit $?
head -22 gpurun_out/launches_all.txt
