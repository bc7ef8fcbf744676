#!/bin/bash
# Round-5 batch 27: per-kernel time of the ResNet-18 step after the conv address / walk changes
# (kernel-trace stats of a short bench run, per-step averages over the 13 steps it runs).
set -o pipefail
O=gpurun_out/${1:-r5_b27}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/trace" -o rn \
  -- python3 bench.py --model resnet18 --steps 10 --warmup 3 --comm-figure off > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:30]:
    print(f'{r["Name"][:70]:70s} calls {int(r["Calls"]):6d} total {float(r["TotalDurationNs"])/1e3:10.1f} us avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
