#!/bin/bash
# GEMM numerics + fprop bench (one-shot / persistent / 16x16x32 configs), then the full GPU suite, smoke()
# and the driver-config headline bench.  usage: bash tools/gpu_r3d.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r3d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gemm.txt 2>&1 || { tail -40 $O/pytest_gemm.txt; exit 1; }
tail -2 $O/pytest_gemm.txt
timeout -k 10 300 python -u tools/gemm_own_bench.py --only fprop,dgrad --out $O/gemm_fprop.jsonl > $O/gemm_fprop.log 2>&1 || { tail -20 $O/gemm_fprop.log; exit 1; }
cut -c1-330 $O/gemm_fprop.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
cut -c1-300 $O/bench_driver.json
