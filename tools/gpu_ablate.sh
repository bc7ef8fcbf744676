#!/bin/bash
# conv backward v2 ablation: phase timelines with W only / D only / both.
set -o pipefail
O=gpurun_out/${1:-ablate}
mkdir -p $O
for d in 0 1 2; do
  timeout -k 10 200 python tools/lenet_phases.py --reps 5 --bwd-dbg $d > $O/phases_dbg$d.txt 2>&1 || exit $?
done
grep conv_bwd $O/phases_dbg*.txt
