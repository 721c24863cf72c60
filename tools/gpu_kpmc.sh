# PMC counters per kernel template instance over ANY python tool (e.g. tools/mlp_micro.py):
# rocprofv3 --pmc passes, each its own run, summarised by tools/pmc_mfma.py (PMC_BY=name)
# -> gpurun_out/kpmc_<tag>.json + a one-line-per-kernel table.
#   bash tools/gpu_kpmc.sh TAG tools/mlp_micro.py [args...]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1
shift
run() {   # run N COUNTERS...
  local n=$1
  shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/kp_$n -o run -- python3 "${CMD[@]}" > gpurun_out/kp_$n.log 2>&1
}
CMD=("$@")
run 1 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT &&
run 2 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE &&
run 3 SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_LDS_DATA_FIFO_FULL GRBM_GUI_ACTIVE
rc=$?
PMC_BY=name python3 tools/pmc_mfma.py gpurun_out/kpmc_$TAG.json $(ls gpurun_out/kp_*/run_results.db 2>/dev/null) > gpurun_out/kpmc_$TAG.txt
cat gpurun_out/kpmc_$TAG.txt
rm -rf gpurun_out/kp_1 gpurun_out/kp_2 gpurun_out/kp_3
exit $rc
