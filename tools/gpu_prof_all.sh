#!/bin/bash
# Kernel profiles (rocprofv3 --kernel-trace --stats) of all three model benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_gpt2" -o gpt2 \
  -- python3 bench.py --model gpt2 --steps 4 --warmup 2 > gpurun_out/prof_gpt2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_rn" -o rn \
  -- python3 bench.py --model resnet18 --steps 4 --warmup 3 > gpurun_out/prof_rn.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o lenet \
  -- python3 bench.py --steps 300 --warmup 20 > gpurun_out/prof.log 2>&1
r=$?
find gpurun_out/prof_gpt2 gpurun_out/prof_rn gpurun_out/prof -name "*kernel_stats.csv"
exit $r
