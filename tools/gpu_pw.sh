# pwgemm change check: pointwise op tests + model steps, bench line, per-launch pwgemm table.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pw or mlp or block or model or configs" > gpurun_out/tpw.log 2>&1; rc=$?
tail -3 gpurun_out/tpw.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/launch_table.py > gpurun_out/launches.txt 2>&1; rc=$?; head -25 gpurun_out/launches.txt; exit $rc
