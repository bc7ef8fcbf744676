#!/usr/bin/env python3
"""Wall / busy time and per-kernel totals of the LAST full training step in a rocprofv3 kernel trace.

usage: python tools/step_window.py <kernel_trace.csv> <step-end kernel substring> [top]
A step is the kernels after one occurrence of the step-end kernel (e.g. the optimizer) up to and
including the next; wall - busy is the GPU idle time inside the step (launch gaps).
"""
import csv
import sys
from collections import defaultdict


def main():
    path, marker = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(idx) < 2:
        sys.exit(f"fewer than two '{marker}' kernels in {path}")
    seg = rows[idx[-2] + 1: idx[-1] + 1]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    busy = sum(dur(r) for r in seg)
    print(f"step: {len(seg)} kernels, wall {wall:.1f} us, busy {busy:.1f} us, idle {wall - busy:.1f} us")
    agg = defaultdict(lambda: [0, 0.0])
    for r in seg:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:80]
        agg[k][0] += 1
        agg[k][1] += dur(r)
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t:9.1f} us {c:4d}x  {k}")


if __name__ == "__main__":
    main()
