# PMC counters per pwgemm template instance over ONE pw_bench case under two knob arms (the
# register-staged and LDS-DMA forms are different template instances): rocprofv3 --pmc passes,
# each its own run, summarised by tools/pmc_mfma.py (PMC_BY=name) -> gpurun_out/pw_pmc.json.
#   bash tools/gpu_pw_pmc.sh "fwd1-gp C512@64" [arm]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CASE=${1:-fwd1-gp C512@64}
ARM=${2:-9=1}
run() {   # run NAME COUNTERS...
  local n=$1
  shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pwp_$n -o run -- python3 tools/pw_bench.py --only "$CASE" --arm "" --arm "$ARM" --rounds 2 --it 5 > gpurun_out/pwp_$n.log 2>&1
}
run 1 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT &&
run 2 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE &&
run 3 SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES GRBM_GUI_ACTIVE &&
run 4 SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_IFETCH_LEVEL GRBM_GUI_ACTIVE &&
run 5 FETCH_SIZE &&
run 6 WRITE_SIZE
rc=$?
PMC_BY=name python3 tools/pmc_mfma.py gpurun_out/pw_pmc.json $(ls gpurun_out/pwp_*/run_results.db 2>/dev/null)
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/pw_pmc.json"))["families"]
for k, v in d.items():
    if "pwgemm" in k:
        print(k)
        print("  " + " ".join("%s=%s" % (a, b) for a, b in v.items()))
PY
rm -rf gpurun_out/pwp_1 gpurun_out/pwp_2 gpurun_out/pwp_3 gpurun_out/pwp_4 gpurun_out/pwp_5 gpurun_out/pwp_6
exit $rc
