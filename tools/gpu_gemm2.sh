#!/bin/bash
# GEMM numerics (all configs incl. the persistent ones on multi-tile shapes) + GPT-2 GEMM bench.
# usage: bash tools/gpu_gemm2.sh <tag> [bench-only-kinds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-gemm2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gemm.txt 2>&1 || { tail -40 $O/pytest_gemm.txt; exit 1; }
tail -2 $O/pytest_gemm.txt
timeout -k 10 600 python -u tools/gemm_own_bench.py --only ${2:-fprop,dgrad,wgrad} --out $O/gemm_bench.jsonl > $O/gemm_bench.log 2>&1 || { tail -20 $O/gemm_bench.log; exit 1; }
cut -c1-420 $O/gemm_bench.jsonl
