#!/bin/bash
# Round-4: driver-config window (--steps 20 --warmup 5) with the first L steps as 1-step graph launches
# (the host submits the long graph under the first step) -- L = 0 / 1 / 2, interleaved, 3 reps.
set -o pipefail
O=gpurun_out/${1:-r4_lead}
mkdir -p $O
for r in 1 2 3; do
  for L in 0 1 2; do
    PDE_BENCH_TRACE=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --comm-figure off --lead-steps $L \
      > $O/L${L}_$r.json 2> $O/L${L}_$r.err || { tail -20 $O/L${L}_$r.err; exit 1; }
    echo "L=$L r=$r $(python3 -c "import json;d=json.load(open('$O/L${L}_$r.json'));print(d['ms_per_step'], d['config']['mode'])") $(grep trace_ $O/L${L}_$r.err)"
  done
done
