#!/bin/bash
# Conv kernels quick loop: numerics tests, per-layer timing, one PMC pass (instruction mix).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1 || { tail -30 gpurun_out/pytest_conv.log; exit 1; }
tail -2 gpurun_out/pytest_conv.log
timeout -k 10 300 python -u tools/conv_bench.py --stages 2 > gpurun_out/conv_bench.jsonl 2> gpurun_out/conv_bench.err || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmc_q" -o conv \
  --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
  -- python3 tools/conv_bench.py --iters 3 --stages 2 > gpurun_out/pmc_q.log 2>&1
