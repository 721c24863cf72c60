# Isolated A/B of the 256-row pwgemm M tiles (DSGAN_PW_BM256=0/1) on the eligible step shapes.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/pw256.log
for e in 0 1; do
  for shp in "fwd 16 512 64 2048" "fwd 16 1024 32 4096" "dgrad 16 1024 32 4096" "dgrad 16 2048 64 256" "fwd 16 256 128 1024" "dgrad 16 256 128 1024"; do
    set -- $shp
    echo -n "BM256=$e " >> gpurun_out/pw256.log
    DSGAN_PW_BM256=$e timeout -k 10 60 python tools/gemm_micro.py $1 $2 $3 $4 $5 1 1 30 bf16 >> gpurun_out/pw256.log 2>&1 || exit 1
  done
done
cat gpurun_out/pw256.log
