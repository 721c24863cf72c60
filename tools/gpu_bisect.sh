# Run one test file/-k selection under several environment settings (A/B bisection of a failure).
#   bash tools/gpu_bisect.sh <testfile[::k]> "ENV=1 ENV2=0" "ENV=0" ...
# Each arm's result goes to gpurun_out/bisect_<i>.txt; a GPU fault, abort or time limit ends the call.
set -o pipefail
sel=$1; shift
i=0
for arm in "$@"; do
  i=$((i + 1))
  env $arm bash tools/gpu_run.sh "testfile=$sel" > gpurun_out/bisect_$i.txt 2>&1
  rc=$?
  for f in gpurun_out/gpu_tests_*.txt; do [ -f "$f" ] && mv "$f" "gpurun_out/bisect_${i}_$(basename "$f")"; done
  echo "arm $i [$arm]: rc=$rc $(grep -E '^(FAILED|=+ .*(passed|failed))' gpurun_out/bisect_$i.txt | tail -1)"
  grep -E "^E |TMPDIAG" gpurun_out/bisect_$i.txt | head -24
  case $rc in 0|1) ;; *) echo "stopping: rc=$rc"; exit $rc ;; esac
done
