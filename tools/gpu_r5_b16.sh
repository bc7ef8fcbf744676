#!/bin/bash
# Round-5 batch 16: HIP graph-launch knobs on the headline window (driver config, comm figure off),
# interleaved reps on one box: default vs DEBUG_HIP_GRAPH_BATCH_SIZE / DEBUG_CLR_MAX_BATCH_SIZE /
# DEBUG_HIP_FORCE_GRAPH_QUEUES settings.
set -o pipefail
O=gpurun_out/${1:-r5_b16}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$AB_VARS" ]; then read -r -a VARS <<< "$AB_VARS"; else
VARS=("NONE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=4" "DEBUG_HIP_GRAPH_BATCH_SIZE=16"
      "DEBUG_HIP_GRAPH_BATCH_SIZE=64" "DEBUG_CLR_MAX_BATCH_SIZE=4" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1"); fi
for r in $(seq 1 ${AB_REPS:-3}); do
  for e in "${VARS[@]}"; do
    env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/v.json 2>> $O/err.txt \
      || { tail -20 $O/err.txt; exit 1; }
    echo "$e rep $r: $(python -c "import json;d=json.load(open('$O/v.json'));print(d['value'], d['ms_per_step'])")" | tee -a $O/summary.txt
  done
done
