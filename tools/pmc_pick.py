#!/usr/bin/env python3
"""Mean PMC counter values per dispatch for kernels whose name contains one of the given substrings.

usage: python tools/pmc_pick.py <dir with */*counter_collection.csv> substr [substr ...]
"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    root, keys = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for p in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            for k in keys:
                if k in r["Kernel_Name"]:
                    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in keys:
        d = acc.get(k, {})
        print(k, {c: f"{sum(v) / len(v):.3g}" for c, v in sorted(d.items())})


if __name__ == "__main__":
    main()
