# Isolated A/B of 256-row WGRAD tiles (DSGAN_PW_BM256_WG=0/1); then the wide-shape parity tests with it on.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/pw256wg.log
for e in 0 1; do
  for shp in "16 1024 32 4096" "16 512 64 2048" "16 256 128 1024" "16 2048 16 1024"; do
    set -- $shp
    echo -n "WG256=$e " >> gpurun_out/pw256wg.log
    DSGAN_PW_BM256_WG=$e timeout -k 10 60 python tools/gemm_micro.py wgrad $1 $2 $3 $4 1 1 30 bf16 2>&1 | grep -v amdgpu.ids >> gpurun_out/pw256wg.log || exit 1
  done
done
cat gpurun_out/pw256wg.log
DSGAN_PW_BM256_WG=1 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "pw_mlp or conv2d" > gpurun_out/t8.log 2>&1; rc=$?; tail -2 gpurun_out/t8.log; exit $rc
