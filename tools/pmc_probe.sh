# PMC counter passes over one contraction (tools/op_micro.py OP): wave/issue/LDS counters, then HBM bytes.
set -o pipefail
OP=${1:-convt}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/op_micro.py $OP > gpurun_out/pm_$OP.log 2>&1 && cat gpurun_out/pm_$OP.log | grep TF &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d gpurun_out/pmc1_$OP -o run --kernel-trace -- python3 tools/op_micro.py $OP 5 > gpurun_out/pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc2_$OP -o run --kernel-trace -- python3 tools/op_micro.py $OP 5 > gpurun_out/pmc2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d gpurun_out/pmc3_$OP -o run --kernel-trace -- python3 tools/op_micro.py $OP 5 > gpurun_out/pmc3.log 2>&1; echo done
