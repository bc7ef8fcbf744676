#!/bin/bash
# Round-5 batch 17: stall-profile PMC over the ResNet-18 step (eager, 2 steps), two SQ groups, summarised
# for the stem / pool / layer-1 kernels.
set -o pipefail
O=gpurun_out/${1:-r5_b17}
mkdir -p $O
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/g$i" -o rn --pmc $grp \
      -- python3 bench.py --model resnet18 --steps 2 --warmup 1 --model-graph off --comm-figure off > $O/g$i.log 2>&1 \
      || { echo "group $i failed"; tail -5 $O/g$i.log; exit 1; }
done
python3 tools/pmc_pick.py $O k_stem_fwd k_stem_wgrad k_bnpool_fwd k_bnpool_bwd k_hconv64 k_hwgrad64 "k_hconv<" "k_wgrad<" > $O/pick.txt
cat $O/pick.txt
