# Round-end style GPU pass on the current tree: the whole -m gpu suite, smoke(), the full bench
# line (quality + cpu_baseline legs) -> gpurun_out/{t_new.log, smoke.log, bench_full.log}.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests_new.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 700 python bench.py > gpurun_out/bench_full.log 2>&1; rc=$?
tail -1 gpurun_out/bench_full.log | cut -c1-400
exit $rc
