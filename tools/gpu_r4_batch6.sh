#!/bin/bash
# Round-4 batch 6: where the driver-config (20-step) window loses ~3 us/step against 2000 steps
# (PDE_BENCH_TRACE host-launch / GPU-event / wall split), and conv_bwd2 role ablations (phase stamps
# with the W or the D role switched off) to see whether the two roles slow each other's load phase.
set -o pipefail
O=gpurun_out/${1:-r4_b6}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  PDE_BENCH_TRACE=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --comm-figure off > $O/w20_$r.json 2> $O/w20_$r.err || { tail -20 $O/w20_$r.err; exit 1; }
done
PDE_BENCH_TRACE=1 timeout -k 10 200 python3 bench.py --steps 200 --warmup 5 --comm-figure off > $O/w200.json 2> $O/w200.err || { tail -20 $O/w200.err; exit 1; }
PDE_BENCH_TRACE=1 timeout -k 10 200 python3 bench.py --steps 2000 --warmup 5 --comm-figure off > $O/w2000.json 2> $O/w2000.err || { tail -20 $O/w2000.err; exit 1; }
for f in w20_1 w20_2 w20_3 w200 w2000; do
  echo "$f $(python3 -c "import json;print(json.load(open('$O/$f.json'))['ms_per_step'])") $(grep trace_ $O/$f.err)"
done
for d in 0 1 2; do
  timeout -k 10 200 python3 tools/lenet_phases.py --bwd-dbg $d > $O/phases_dbg$d.txt 2>&1 || { tail -20 $O/phases_dbg$d.txt; exit 1; }
  echo "dbg=$d"; grep conv_bwd $O/phases_dbg$d.txt | cut -c1-600
done
