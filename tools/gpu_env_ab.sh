# Same-box bench A/B of an environment toggle, alternating: bash tools/gpu_env_ab.sh VAR   (VAR=1 vs VAR=0)
set -o pipefail
for v in 1 0 1 0; do
  env "$1=$v" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-quality --no-train-equiv > gpurun_out/env_ab.log 2>&1 || exit 1
  echo "$1=$v $(tail -1 gpurun_out/env_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
