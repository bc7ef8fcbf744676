#!/usr/bin/env python3
"""Average PMC counter value per dispatch, per kernel, from rocprofv3 counter_collection.csv files."""
import csv
import sys
from collections import defaultdict


def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:28]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    keys = sorted({c for k in acc for c in acc[k]})
    kern = [k for k in acc if k.startswith("k_")]
    print("| counter | " + " | ".join(kern) + " |")
    print("|---|" + "---|" * len(kern))
    for c in keys:
        vals = []
        for k in kern:
            v = acc[k].get(c)
            vals.append(f"{sum(v) / len(v):.4g}" if v else "")
        print(f"| {c} | " + " | ".join(vals) + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
