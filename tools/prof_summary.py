#!/usr/bin/env python3
"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into a markdown table (for ``profiles/``).

usage: python tools/prof_summary.py gpurun_out/prof/lenet_kernel_stats.csv [title] [steps]
"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    m = re.match(r"(?:void )?([\w:<>, ]+?)\(", name)
    base = m.group(1) if m else name
    return base[:90]


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else None
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"## {title}\n")
    print(f"source: `{path}` (rocprofv3 --kernel-trace --stats)\n")
    hdr = "| kernel | calls | avg µs | min µs | max µs | % of GPU time |" + (" µs / step |" if steps else "")
    print(hdr)
    print("|" + "---|" * (hdr.count("|") - 1))
    for r in rows:
        line = (f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                f"{float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | {float(r['Percentage']):.2f} |")
        if steps:
            line += f" {float(r['TotalDurationNs']) / 1e3 / steps:.2f} |"
        print(line)
    print(f"\ntotal kernel time: {total / 1e6:.2f} ms" + (f" ({total / 1e3 / steps:.2f} µs per step)" if steps else ""))


if __name__ == "__main__":
    main()
