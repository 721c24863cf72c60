set -o pipefail
mkdir -p gpurun_out
for t in 128 256 -1; do echo "tile $t"; DSGAN_PW_FD_TILE=$t timeout -k 10 120 python tools/pwdgrad_micro.py 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/pwtile2.log
cat gpurun_out/pwtile2.log
