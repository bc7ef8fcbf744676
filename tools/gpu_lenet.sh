#!/bin/bash
# LeNet headline session: GPU tests of the fused step, then bench variants (+ rocprof stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_lenet_gpu.py tests/test_ops_gpu.py -q > gpurun_out/pytest_lenet.log 2>&1; r=$?
tail -15 gpurun_out/pytest_lenet.log
[ $r -le 1 ] || exit $r
for mode in "--mode graph --graph-steps 10" "--mode graph --graph-steps 1" "--mode eager"; do
  timeout -k 10 300 python bench.py --steps 2000 --warmup 200 $mode >> gpurun_out/bench_lenet_variants.jsonl 2>> gpurun_out/bench_lenet.err || exit 1
done
cat gpurun_out/bench_lenet_variants.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o lenet \
    -- python3 bench.py --steps 300 --warmup 20 > gpurun_out/prof.log 2>&1
echo "rc=$?"
