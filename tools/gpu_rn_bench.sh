#!/bin/bash
# ResNet-18 bench + kernel trace of a short run (per-step breakdown by tools/step_breakdown.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/bench_resnet18.json 2> gpurun_out/bench_resnet18.err && cat gpurun_out/bench_resnet18.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/prof_rn" -o rn \
  -- python3 bench.py --model resnet18 --steps 4 --warmup 3 > gpurun_out/prof_rn.log 2>&1
