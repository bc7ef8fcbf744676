#!/bin/bash
# PMC counter passes over the eager LeNet v2 step (each --pmc group in its own run; no trace domains).
set -o pipefail
O=gpurun_out/${1:-pmc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/g$i" -o lenet --pmc $grp \
      -- python3 bench.py --steps 40 --warmup 5 --mode eager --comm-figure off > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -5 $O/g$i.log; }
done
python3 tools/pmc_summary.py $(find $O -name "*counter_collection.csv") > $O/summary.md 2>&1
cat $O/summary.md
