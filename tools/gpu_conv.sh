#!/bin/bash
# Conv kernels session: numerics tests, per-layer timing vs MIOpen, ResNet-18 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_resnet_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1; r=$?
tail -25 gpurun_out/pytest_conv.log
[ $r -le 1 ] || exit $r
timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/conv_bench.jsonl 2> gpurun_out/conv_bench.err || exit $?
cat gpurun_out/conv_bench.jsonl
timeout -k 10 300 python bench.py --model resnet18 --steps 10 --warmup 3 > gpurun_out/bench_resnet.json 2> gpurun_out/bench_resnet.err || exit $?
cat gpurun_out/bench_resnet.json
exit $r
