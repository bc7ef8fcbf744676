#!/bin/bash
# GPT-2 small: bench + kernel profile (rocprofv3 --kernel-trace --stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --model gpt2 --steps 10 --warmup 3 > gpurun_out/bench_gpt2.json 2> gpurun_out/bench_gpt2.err || exit $?
cat gpurun_out/bench_gpt2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_gpt2" -o gpt2 \
  -- python3 bench.py --model gpt2 --steps 4 --warmup 2 > gpurun_out/prof_gpt2.log 2>&1
