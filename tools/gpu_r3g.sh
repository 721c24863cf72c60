# PMC passes only: HBM traffic per family + MFMA/LDS/issue counters per family -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_pmc.sh || exit $?
rm -rf gpurun_out/pmcf gpurun_out/pmcw
bash tools/gpu_mfma_pmc.sh || exit $?
