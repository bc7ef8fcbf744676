#!/usr/bin/env python3
"""Per-step kernel durations over a long rocprofv3 kernel trace of the LeNet bench: median duration of
every kernel per window of steps (a step starts at each k_conv_fwd2 dispatch), to locate a slowdown
that appears only at some points of a run.

    python tools/step_drift.py <kernel_trace.csv> [--window 500]
"""
import argparse
import csv
import statistics


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0][:24]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=int, default=500)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        k = short(r["Kernel_Name"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if k.startswith("k_conv_fwd2"):
            cur = {"t0": s, "k": {}}
            steps.append(cur)
        if cur is not None:
            cur["k"][k] = cur["k"].get(k, 0) + (e - s) / 1e3
            cur["t1"] = e
    names = sorted({k for st in steps for k in st["k"]})
    print("steps", len(steps))
    print(f"{'window':>12s} {'span_us':>8s} " + " ".join(f"{n[:12]:>12s}" for n in names))

    def line(lbl, ws):
        span = statistics.median([(ws[i + 1]["t0"] - ws[i]["t0"]) / 1e3 for i in range(len(ws) - 1)]) if len(ws) > 1 else 0
        cols = [statistics.median([st["k"].get(n, 0) for st in ws]) for n in names]
        print(f"{lbl:>12s} {span:8.2f} " + " ".join(f"{c:12.2f}" for c in cols))
    for i in range(0, len(steps), a.window):
        line(f"{i}", steps[i:i + a.window])
    line("last25", steps[-25:])


if __name__ == "__main__":
    main()
