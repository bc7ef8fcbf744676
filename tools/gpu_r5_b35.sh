#!/bin/bash
# Round-5 batch 35: per-kernel time of the GPT-2 step with the final round-5 kernels (kernel-trace stats
# of a short bench run; per-step figures = totals / steps run).
set -o pipefail
O=gpurun_out/${1:-r5_b35}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/trace" -o g \
  -- python3 bench.py --model gpt2 --steps 8 --warmup 2 --comm-figure off > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:28]:
    print(f'{r["Name"][:70]:70s} calls {int(r["Calls"]):6d} total {float(r["TotalDurationNs"])/1e3:10.1f} us avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
