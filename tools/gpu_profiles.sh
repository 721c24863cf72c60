# All profile artifacts of the current tree: rocprofv3 kernel stats, PMC HBM traffic, MFMA/LDS
# counters, the per-launch HIP-event table -> gpurun_out/ (copy the ones to keep to profiles/).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_prof.sh || exit $?
bash tools/gpu_pmc.sh || exit $?
rm -rf gpurun_out/pmcf gpurun_out/pmcw
bash tools/gpu_mfma_pmc.sh || exit $?
timeout -k 10 200 python tools/launch_table.py > gpurun_out/launches_all.txt 2>&1
