#!/bin/bash
# Round 6 final build: kernel trace + per-kernel stats of the toy-CNN headline (graph replay, comm off),
# a step timeline from mid-run and the kernel-to-kernel gaps.
set -o pipefail
O=gpurun_out/${1:-r6_ltrace}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof" -o l -- \
  python3 bench.py --steps 200 --warmup 10 --comm-figure off > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
T=$(ls $O/prof/*kernel_trace.csv | head -n 1)
python3 tools/trace_summary.py "$T" k_conv_fwd2 14 > $O/timeline.txt
python3 - "$T" > $O/gaps.txt <<'PY'
import csv, sys, statistics
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nm = lambda r: r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]
gaps = {}
for a, b in zip(rows, rows[1:]):
    gaps.setdefault(nm(a) + " -> " + nm(b), []).append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000)
for k, v in sorted(gaps.items(), key=lambda x: -len(x[1])):
    if len(v) >= 20: print(f"gap {k:85s} median {statistics.median(v):6.2f} us x{len(v)}")
PY
cp $O/prof/*kernel_stats.csv $O/kernel_stats.csv
rm -f $O/prof/*kernel_trace.csv
cat $O/timeline.txt $O/gaps.txt
