# per-dispatch kernel trace of one bench step + depthwise micro timings -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_prof.sh || exit 1
tail -1 gpurun_out/prof_top.txt
head -1 gpurun_out/prof_dispatch.csv
timeout -k 10 120 python3 tools/dw_micro.py > gpurun_out/dw_micro.txt 2>&1 || { tail -5 gpurun_out/dw_micro.txt; exit 1; }
cat gpurun_out/dw_micro.txt
