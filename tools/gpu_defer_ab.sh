set -o pipefail
for d in 1 0 1 0; do
  DSGAN_DEFER_SPLITS=$d timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-quality --no-train-equiv > gpurun_out/ab_$d.log 2>&1 || exit 1
  echo "defer=$d $(tail -1 gpurun_out/ab_$d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-quality --no-train-equiv > gpurun_out/prof.log 2>&1 || exit 1
python3 tools/prof_stats.py gpurun_out/prof/run_results.db gpurun_out/prof_stats.csv --steps 15 > gpurun_out/prof_top.txt 2>&1
python3 tools/prof_dispatch.py gpurun_out/prof/run_results.db gpurun_out/prof_dispatch.csv --last 786 || true
rm -rf gpurun_out/prof
