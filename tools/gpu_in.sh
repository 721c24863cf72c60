set -o pipefail
mkdir -p gpurun_out
for m in 0 1 2; do DSGAN_IN_V4=$m timeout -k 10 120 python tools/in_micro.py >> gpurun_out/in.log 2>&1 || exit $?; done
