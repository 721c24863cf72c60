# MFMA / issue / LDS counters per kernel over a short bench run: rocprofv3 --pmc passes, each its own
# run (MI355X_MICROARCH.md § rocprofv3 PMC slots: <= 8 SQ, 2 GRBM per pass), summarised on the box
# (tools/pmc_mfma.py) -> gpurun_out/mfma_pmc.json; the result databases are deleted (size).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-quality --no-train-equiv"
timeout -s KILL 30 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1
echo "list rc=$?"
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/mfma_pmc1 -o run -- $B > gpurun_out/mfma_pmc1.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/mfma_pmc2 -o run -- $B > gpurun_out/mfma_pmc2.log 2>&1
rc=$?
echo "pmc rc=$rc"
ls -la gpurun_out/mfma_pmc1 gpurun_out/mfma_pmc2 2>&1 | head -20
python3 tools/pmc_mfma.py gpurun_out/mfma_pmc.json $(ls gpurun_out/mfma_pmc*/run_results.db 2>/dev/null)
rm -rf gpurun_out/mfma_pmc1 gpurun_out/mfma_pmc2
exit $rc
