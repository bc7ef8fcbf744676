#!/bin/bash
# Attention kernels: numerics tests, timing, one PMC pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -q -k "attention or gpt2" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1 || { tail -30 gpurun_out/pytest_attn.log; exit 1; }
tail -2 gpurun_out/pytest_attn.log
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_bench.json 2> gpurun_out/attn_bench.err || exit $?
cat gpurun_out/attn_bench.json
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmc_attn" -o attn \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU \
  -- python3 tools/attn_bench.py --iters 3 > gpurun_out/pmc_attn.log 2>&1
