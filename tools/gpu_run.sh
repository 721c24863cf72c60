# One parameterised GPU session on the gpurun box (replaces the per-call tools/gpu_r3*.sh scripts).
#
#   bash tools/gpu_run.sh STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the first failing step ends the call (a GPU
# fault, abort or time limit leaves nothing else running on the card).  Outputs go to gpurun_out/.
#   tests[=<pytest -k expr>]  the -m gpu suite, or the subset -k selects (+ for spaces) -> gpu_tests.txt
#   testfile=<path>[::k]      one test file (optionally -k)                 -> gpu_tests_<name>.txt
#   smoke                     __graft_entry__.smoke()                       -> smoke.txt
#   bench[=<bench.py args>]   the bench line ('+' separates arguments)       -> bench.log
#   nan[=<arm,arm,...>]       tools/nan_diag.py (default arms base,fold)    -> nan_diag.txt
#   pwbench[=<arm/arm/...>]   tools/pw_bench.py planner-knob A/B ("base" = built-in knobs,
#                             an arm is k=v[,k=v])                          -> pw_bench.txt
#   launches                  tools/launch_table.py per-launch HIP-event table -> launches_all.txt
#   prof                      rocprofv3 kernel stats of a short bench run (tools/gpu_prof.sh)
#   pmc                       PMC HBM traffic + MFMA/LDS counters (tools/gpu_pmc.sh, gpu_mfma_pmc.sh)
#   pwpmc=<case>[/arm]        per-instance PMC of one pw_bench case ('+' for spaces), two arms (tools/gpu_pw_pmc.sh)
#   kpmc=<tag>:<script>[+args] per-kernel-instance PMC over a python tool (tools/gpu_kpmc.sh)
#   py=<script>[+args]        any python tool under tools/ (limit 600 s)     -> <script>.txt
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1

run() {   # run LIMIT LOG CMD... : the step's output to LOG; on failure print its tail and stop
  local lim=$1 log=$2
  shift 2
  echo "== $(date +%T) $*" | cut -c1-200
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "step failed rc=$rc: $*" | cut -c1-200
    tail -40 "$log"
    exit $rc
  fi
}

for step in "$@"; do
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  case "$name" in
    tests)
      if [ -n "$arg" ]; then
        run 1200 gpurun_out/gpu_tests.txt python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "${arg//+/ }"
      else
        run 1200 gpurun_out/gpu_tests.txt python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
      fi
      tail -2 gpurun_out/gpu_tests.txt ;;
    testfile)
      f=${arg%%::*}; k=""
      [ "$f" != "$arg" ] && k=${arg#*::} && k=${k//+/ }
      log=gpurun_out/gpu_tests_$(basename "$f" .py).txt
      if [ -n "$k" ]; then
        run 1200 "$log" python -u -m pytest "$f" -m gpu -x -v -s --timeout 1100 --timeout-method thread -k "$k"
      else
        run 1200 "$log" python -u -m pytest "$f" -m gpu -x -v -s --timeout 1100 --timeout-method thread
      fi
      grep -E "^(C[0-9]|peak)|passed|failed" "$log" | tail -8 ;;
    smoke)
      run 300 gpurun_out/smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
      tail -1 gpurun_out/smoke.txt ;;
    bench)
      # shellcheck disable=SC2086
      run 900 gpurun_out/bench.log python -u bench.py ${arg//+/ }
      tail -1 gpurun_out/bench.log | cut -c1-400 ;;
    nan)
      # shellcheck disable=SC2086
      run 900 gpurun_out/nan_diag.txt python -u tools/nan_diag.py ${arg//,/ }
      grep -vE "UserWarning|Consider using|vals = dict" gpurun_out/nan_diag.txt | tail -60 ;;
    pwbench)
      args=()
      IFS='/' read -ra arms <<< "${arg:-base/0=0}"
      for a in "${arms[@]}"; do [ "$a" = base ] && a=""; args+=(--arm "$a"); done
      run 600 gpurun_out/pw_bench.txt python -u tools/pw_bench.py "${args[@]}"
      tail -45 gpurun_out/pw_bench.txt ;;
    launches)
      run 300 gpurun_out/launches_all.txt python tools/launch_table.py
      head -30 gpurun_out/launches_all.txt ;;
    prof)
      bash tools/gpu_prof.sh || exit $?
      tail -3 gpurun_out/prof_top.txt ;;
    pmc)
      bash tools/gpu_pmc.sh || exit $?
      rm -rf gpurun_out/pmcf gpurun_out/pmcw
      bash tools/gpu_mfma_pmc.sh || exit $? ;;
    pwpmc)
      c=${arg%%/*}; arm="9=1"
      [ "$c" != "$arg" ] && arm=${arg#*/}
      c=${c//+/ }
      timeout -k 10 900 bash tools/gpu_pw_pmc.sh "$c" "$arm" > gpurun_out/pw_pmc.txt 2>&1 || { tail -30 gpurun_out/pw_pmc.txt; exit 1; }
      tail -12 gpurun_out/pw_pmc.txt ;;
    kpmc)
      tag=${arg%%:*}; sc=${arg#*:}; s=${sc%%+*}; rest=""
      [ "$s" != "$sc" ] && rest=${sc#*+}
      # shellcheck disable=SC2086
      timeout -k 10 900 bash tools/gpu_kpmc.sh "$tag" "tools/$s" ${rest//+/ } > gpurun_out/kpmc_run_$tag.txt 2>&1 || { tail -30 gpurun_out/kpmc_run_$tag.txt; exit 1; }
      head -25 gpurun_out/kpmc_$tag.txt ;;
    py)
      s=${arg%%+*}; rest=""
      [ "$s" != "$arg" ] && rest=${arg#*+}
      # shellcheck disable=SC2086
      run 600 "gpurun_out/$(basename "$s" .py).txt" python -u "tools/$s" ${rest//+/ }
      tail -40 "gpurun_out/$(basename "$s" .py).txt" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== $(date +%T) all steps done"
