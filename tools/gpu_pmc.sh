# HBM traffic per kernel family: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a short bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-quality --no-train-equiv > gpurun_out/pmcf.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-quality --no-train-equiv > gpurun_out/pmcw.log 2>&1 &&
python3 tools/pmc_traffic.py gpurun_out/pmcf/run_results.db gpurun_out/pmcw/run_results.db gpurun_out/pmc_traffic.json
