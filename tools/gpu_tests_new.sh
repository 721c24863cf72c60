# GPU pass over the given pytest arguments (default: the whole -m gpu suite), one pytest process.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ $# -eq 0 ]; then set -- tests; fi
timeout -k 10 1100 python -u -m pytest "$@" -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1
rc=$?
tail -30 gpurun_out/t_new.log
exit $rc
