# pconv BM=256 vs 128 at the VGG conv3/conv4 shapes (fwd, dgrad), then pconv parity tests
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/pc.log
for bm in 0 1; do
  for args in "fwd 16 256 64 256 3 1" "dgrad 16 256 64 256 3 1" "fwd 16 512 32 512 3 1" "dgrad 16 512 32 512 3 1" "fwd 16 256 32 512 3 1" "fwd 16 128 64 256 3 1"; do
    DSGAN_PC_BM256=$bm timeout -k 10 60 python tools/gemm_micro.py $args 20 bf16 >> gpurun_out/pc.log 2>&1 || exit $?
    echo "  (bm256=$bm)" >> gpurun_out/pc.log
  done
done
grep -E "TF/s|bm256" gpurun_out/pc.log | paste - -
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pconv or conv2d or perceptual or full_step" > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; exit $rc
