# in-process A/B of the step's pointwise launches under planner knobs (tools/pw_bench.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pw_bench.py --arm "" --arm "0=0" --arm "2=512" --arm "4=1" --arm "5=1" \
  > gpurun_out/r3h_pwbench.log 2>&1 || { tail -30 gpurun_out/r3h_pwbench.log; exit 1; }
cat gpurun_out/r3h_pwbench.log
