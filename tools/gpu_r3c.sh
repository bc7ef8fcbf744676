#!/bin/bash
# Round-3 session: GEMM numerics + GPT-2 GEMM shapes (one-shot vs persistent), the status pass of
# gpu_session.sh (benches, model step windows, GPU tests) and the graph-steps A/B of the headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r3c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gemm.txt 2>&1 || { tail -30 $O/pytest_gemm.txt; exit 1; }
tail -2 $O/pytest_gemm.txt
timeout -k 10 300 python -u tools/gemm_own_bench.py --only fprop,dgrad --out $O/gemm_bench.jsonl > $O/gemm_bench.log 2>&1 || { tail -20 $O/gemm_bench.log; exit 1; }
cut -c1-300 $O/gemm_bench.jsonl
bash tools/gpu_session.sh ${1:-r3c}/s benches || exit 1
bash tools/gpu_graphsteps.sh ${1:-r3c}/gs 2 || exit 1
bash tools/gpu_session.sh ${1:-r3c}/s prof || exit 1
bash tools/gpu_session.sh ${1:-r3c}/s tests
