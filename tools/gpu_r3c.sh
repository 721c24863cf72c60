# probe + the -m gpu suite + C2 / C5-fp16 bench lines (no CPU legs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/fp16_scale_probe.py 512 8 > gpurun_out/probe.log 2>&1; rc=$?
grep -v "^initialize\|^model\|Vgg16\|amdgpu.ids" gpurun_out/probe.log | head -20; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r3.sh "$@"
