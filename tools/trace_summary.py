#!/usr/bin/env python3
"""Median duration per kernel from a rocprofv3 kernel_trace.csv (+ optional per-step timeline)."""
import csv
import statistics
import sys


def name(r):
    return r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]


def main(path, timeline_from=None, n=8):
    rows = list(csv.DictReader(open(path)))
    d = {}
    for r in rows:
        d.setdefault(name(r), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for k, v in sorted(d.items(), key=lambda x: -statistics.median(x[1]) * len(x[1]))[:15]:
        print(f"{k:60s} median {statistics.median(v):8.2f} us  x{len(v)}")
    if timeline_from:
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        i = len(rows) // 2
        while timeline_from not in name(rows[i]):
            i += 1
        t0 = int(rows[i]["Start_Timestamp"])
        for r in rows[i:i + n]:
            s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
            print(f"  {name(r):30s} {s / 1000:8.2f} -> {e / 1000:8.2f}  ({(e - s) / 1000:6.2f})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None, int(sys.argv[3]) if len(sys.argv) > 3 else 8)
