# GPU pass over the given test files (default: the whole -m gpu suite), one pytest process.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${@:-tests}
timeout -k 10 1100 python -u -m pytest $T -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1
rc=$?
tail -30 gpurun_out/t_new.log
exit $rc
