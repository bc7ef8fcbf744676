#!/bin/bash
# Round-4: kernel-trace timeline of the headline step (kernel start / end as the CP sees them) to
# compare the boundaries with the in-kernel phase stamps.
set -o pipefail
O=gpurun_out/${1:-r4_ltrace}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/prof" -o l -- \
  python3 bench.py --steps 60 --warmup 10 --comm-figure off > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
T=$(ls $O/prof/*kernel_trace.csv | head -n 1)
python3 tools/trace_summary.py "$T" k_conv_fwd2 14 > $O/timeline.txt
python3 - "$T" > $O/gaps.txt <<'PY'
import csv, sys, statistics
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nm = lambda r: r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]
gaps, durs = {}, {}
for a, b in zip(rows, rows[1:]):
    k = nm(a) + " -> " + nm(b)
    gaps.setdefault(k, []).append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000)
for r in rows:
    durs.setdefault(nm(r), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(gaps.items(), key=lambda x: -len(x[1])):
    if len(v) >= 20: print(f"gap {k:85s} median {statistics.median(v):6.2f} us x{len(v)}")
for k, v in sorted(durs.items(), key=lambda x: -len(x[1])):
    if len(v) >= 20: print(f"dur {k:45s} median {statistics.median(v):6.2f} us x{len(v)}")
PY
rm -f $O/prof/*kernel_trace.csv
cat $O/gaps.txt
