#!/bin/bash
# PMC counter passes over the eager LeNet step (each --pmc group in its own run; no trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT" \
           "SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmc2/g$i" -o lenet --pmc $grp \
      -- python3 bench.py --steps 40 --warmup 5 --mode eager > gpurun_out/pmc2/g$i.log 2>&1 || { echo "group $i failed"; tail -5 gpurun_out/pmc2/g$i.log; exit 1; }
done
echo done
