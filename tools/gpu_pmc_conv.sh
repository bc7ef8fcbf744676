#!/bin/bash
# PMC counter passes over the ResNet conv kernels (tools/conv_bench.py, one stage depth), each group
# in its own run; counters only with --kernel-trace (no trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_conv
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmc_conv/g$i" -o conv --pmc $grp \
      -- python3 tools/conv_bench.py --iters 3 --stages 2 > gpurun_out/pmc_conv/g$i.log 2>&1 || { echo "group $i failed"; tail -5 gpurun_out/pmc_conv/g$i.log; exit 1; }
done
echo done
