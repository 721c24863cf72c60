set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
timeout -k 10 120 python tools/op_micro.py convt > gpurun_out/pm.log 2>&1 && cat gpurun_out/pm.log &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d gpurun_out/pmc1 -o run --kernel-trace -- python3 tools/op_micro.py convt 5 > gpurun_out/pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc2 -o run --kernel-trace -- python3 tools/op_micro.py convt 5 > gpurun_out/pmc2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d gpurun_out/pmc3 -o run --kernel-trace -- python3 tools/op_micro.py convt 5 > gpurun_out/pmc3.log 2>&1; echo done
