# Issue / VALU / MFMA / LDS counters per MLP kernel instance over tools/mlp_micro.py (MLP_SHAPES
# selects the block shapes): three rocprofv3 --pmc passes -> gpurun_out/mlp_pmc.json.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 tools/mlp_micro.py"
rm -rf gpurun_out/mlpp1 gpurun_out/mlpp2 gpurun_out/mlpp3
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/mlpp1 -o run -- $B > gpurun_out/mlpp1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/mlpp2 -o run -- $B > gpurun_out/mlpp2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/mlpp3 -o run -- $B > gpurun_out/mlpp3.log 2>&1
rc=$?
echo "pmc rc=$rc"
PMC_BY=name python3 tools/pmc_mfma.py gpurun_out/mlp_pmc.json $(ls gpurun_out/mlpp*/run_results.db 2>/dev/null)
rm -rf gpurun_out/mlpp1 gpurun_out/mlpp2 gpurun_out/mlpp3
exit $rc
