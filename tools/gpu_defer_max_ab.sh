set -o pipefail
for v in "" 8 64 "" 8 64; do
  DSGAN_SPLIT_DEFER_MAX_MB=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-quality --no-train-equiv > gpurun_out/abm.log 2>&1 || exit 1
  echo "max_mb=[$v] $(tail -1 gpurun_out/abm.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
