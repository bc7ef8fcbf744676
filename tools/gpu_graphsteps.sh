#!/bin/bash
# Driver-config headline bench (--steps 20 --warmup 5) with the 20 timed steps launched as graphs of
# 20 / 10 / 5 steps, interleaved on one box.  usage: bash tools/gpu_graphsteps.sh <tag> [reps]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-graphsteps}
REPS=${2:-3}
mkdir -p $O
export TMPDIR=/tmp
: > $O/ab.txt
for r in $(seq 1 $REPS); do
  for g in 20 10 5; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --comm-figure off --graph-steps $g > $O/g$g.$r.json 2> $O/g$g.$r.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/g$g.$r.json')); print('graph_steps=$g rep=$r', d['ms_per_step']*1e3, 'us/step', d['value'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
