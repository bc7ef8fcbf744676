#!/bin/bash
# Round-4 status pass: LeNet phase timelines (defer / fold), driver-config bench, W=1 comm figure.
set -o pipefail
O=gpurun_out/${1:-r4_base}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/lenet_phases.py --reps 5 --json $O/phases.json > $O/phases.txt 2>&1 &&
PDE_LENET_BWD_MODE=fold timeout -k 10 300 python tools/lenet_phases.py --reps 5 > $O/phases_fold.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err &&
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --comm-figure off > $O/bench2000.json 2> $O/bench2000.err
rc=$?
cat $O/phases.txt $O/phases_fold.txt; cut -c1-400 $O/bench20.json $O/bench2000.json
exit $rc
