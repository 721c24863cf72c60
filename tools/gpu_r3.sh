# Round-3 GPU pass: the -m gpu suite (args: pytest selection, default all), then the C2 bench line
# and the C5 fp16 bench line (no CPU legs) -> gpurun_out/{t_new.log, bench_c2.log, bench_c5.log}.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests_new.sh "$@" || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quality > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | cut -c1-300
timeout -k 10 300 python bench.py --size 512 --batch 8 --precision fp16 --no-cpu-baseline --no-quality > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5.log | cut -c1-300
