#!/usr/bin/env python3
"""Per-step kernel breakdown from a rocprofv3 kernel_trace.csv: the last N steps, delimited by a
kernel that runs once per step (default the optimizer), averaged per step.

usage: python tools/step_breakdown.py TRACE.csv [marker_substring] [nsteps] [top]"""
import collections
import csv
import sys


def main(path, marker="k_sgd_master", nsteps=3, top=25):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(idx) < nsteps + 1:
        raise SystemExit(f"only {len(idx)} '{marker}' kernels in the trace")
    seg = rows[idx[-nsteps - 1] + 1: idx[-1] + 1]
    wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3 / nsteps
    d, c = collections.defaultdict(float), collections.Counter()
    for r in seg:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:80]
        d[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / nsteps
        c[n] += 1
    print(f"| kernel | launches / step | us / step |\n|---|---|---|")
    for n, v in sorted(d.items(), key=lambda x: -x[1])[:top]:
        print(f"| `{n}` | {c[n] // nsteps} | {v:.1f} |")
    print(f"\nsum of kernel time {sum(d.values()):.1f} us / step; wall {wall:.1f} us / step "
          f"(last {nsteps} steps of `{path}`)")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1] if len(a) > 1 else "k_sgd_master", int(a[2]) if len(a) > 2 else 3,
         int(a[3]) if len(a) > 3 else 25)
