# Round-3 profile pass: rocprof stats + PMC traffic + MFMA/LDS counters + launch table of the C2
# bench (tools/gpu_profiles.sh), then the C5 fp16 bench line WITH its MS-SSIM quality leg and CPU
# baseline (512^2, batch 8) -> gpurun_out/bench_c5q.log
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_profiles.sh || exit $?
timeout -k 10 780 python bench.py --size 512 --batch 8 --precision fp16 > gpurun_out/bench_c5q.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5q.log | cut -c1-300
