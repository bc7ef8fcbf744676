#!/bin/bash
# Own GEMM session: numerics tests, then the GPT-2 GEMM bench (own configs vs hipBLASLt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gemm
export TMPDIR=/tmp
STAGE=${1:-all}
tests() { timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm/pytest.log 2>&1; r=$?; tail -30 gpurun_out/gemm/pytest.log; return $r; }
bench() { timeout -k 10 600 python -u tools/gemm_own_bench.py --out gpurun_out/gemm/bench.jsonl ${BENCH_ARGS:-} > gpurun_out/gemm/bench.log 2>&1; r=$?; cat gpurun_out/gemm/bench.log | cut -c1-400; return $r; }
case "$STAGE" in
  tests) tests ;;
  bench) bench ;;
  all) tests && bench ;;
esac
rc=$?
echo "stage=$STAGE rc=$rc"
exit $rc
