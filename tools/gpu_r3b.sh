# fp16 loss-scale probe at C5, then the -m gpu suite (args: pytest selection) -> gpurun_out/{probe.log,t_new.log}
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/fp16_scale_probe.py 512 8 > gpurun_out/probe.log 2>&1; rc=$?
cat gpurun_out/probe.log | grep -v "^initialize\|^model\|Vgg16" ; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_tests_new.sh "$@"
