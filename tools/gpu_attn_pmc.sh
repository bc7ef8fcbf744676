#!/bin/bash
# Attention kernels at the GPT-2 shape: timing (tools/attn_bench.py) then PMC passes, one counter
# group per rocprofv3 run (no trace domains), summarised per kernel into OUT/pmc.md.
set -o pipefail
OUT=gpurun_out/${1:-attn_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/attn_bench.py --variants ${VARIANTS:-5} > $OUT/bench.jsonl 2> $OUT/bench.err || exit 1
cat $OUT/bench.jsonl
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/g$i" -o pmc --pmc $grp \
      -- python3 tools/attn_bench.py --iters 2 --variants 5 > $OUT/g$i.log 2>&1 || { echo "group $i failed"; tail -5 $OUT/g$i.log; exit 1; }
done
python tools/pmc_pick.py $OUT k_attn_fwd k_attn_bwd_dq k_attn_bwd_dkdv > $OUT/pmc.md
cat $OUT/pmc.md
