#!/bin/bash
# PMC counter passes over the ResNet-18 bench (eager steps: graph replay off so every dispatch is
# attributed): one counter group per rocprofv3 run, no trace domains.  Summary per kernel (mean per
# dispatch) in gpurun_out/<tag>/summary.md.  usage: bash tools/gpu_pmc_resnet.sh <tag>
set -o pipefail
O=gpurun_out/${1:-pmc_rn}
mkdir -p $O
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/g$i" -o rn --pmc $grp \
      -- python3 bench.py --model resnet18 --steps 2 --warmup 1 --model-graph off > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -5 $O/g$i.log; exit 1; }
done
python3 tools/pmc_summary.py $(find $O -name "*counter_collection.csv") > $O/summary.md 2>&1
cat $O/summary.md
