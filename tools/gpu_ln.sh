#!/bin/bash
# LayerNorm-backward rework: numerics tests, GPT-2 bench, kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tf.log 2>&1 || { tail -30 gpurun_out/pytest_tf.log; exit 1; }
tail -2 gpurun_out/pytest_tf.log
bash tools/gpu_gptprof.sh || exit $?
f=$(ls gpurun_out/prof_gpt2/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && python tools/prof_summary.py "$f" "GPT-2 W=1" 6 > gpurun_out/gpt2_kernel_stats.md && head -30 gpurun_out/gpt2_kernel_stats.md
