#!/usr/bin/env python3
"""Per-step GPU time of the timed window in a rocprofv3 kernel trace of ``bench.py`` (toy CNN).

usage: python tools/window_steps.py <kernel_trace.csv> [steps] [kernels_per_step]
The last ``steps`` x ``kernels_per_step`` step kernels (k_conv_fwd2 ... k_adam) are the timed window;
prints each step's span (conv forward start -> next conv forward start; the last step to its Adam
end), the kernels' durations, and the idle time between the window's steps and before its first.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    kps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if "k_" in r["Kernel_Name"] and "lenet" not in r["Kernel_Name"].lower()
          and any(n in r["Kernel_Name"] for n in ("k_conv_fwd2", "k_fc1_fwd", "k_head2", "k_fc_bwd",
                                                  "k_conv_bwd2", "k_adam"))]
    win = ks[-steps * kps:]
    if len(win) < steps * kps:
        sys.exit("not enough step kernels in the trace")
    t = lambda r, k: int(r[k]) / 1e3
    starts = [t(win[i * kps], "Start_Timestamp") for i in range(steps)]
    end = t(win[-1], "End_Timestamp")
    prev = ks[-steps * kps - 1] if len(ks) > steps * kps else None
    if prev is not None:
        print(f"idle before the window: {starts[0] - t(prev, 'End_Timestamp'):.2f} us")
    tot = end - starts[0]
    print(f"window: {tot:.1f} us GPU, {tot / steps:.2f} us/step")
    for i in range(steps):
        e = starts[i + 1] if i + 1 < steps else end
        ds = [t(r, "End_Timestamp") - t(r, "Start_Timestamp") for r in win[i * kps:(i + 1) * kps]]
        print(f"step {i:2d}: {e - starts[i]:7.2f} us  kernels " + " ".join(f"{d:6.2f}" for d in ds))


if __name__ == "__main__":
    main()
