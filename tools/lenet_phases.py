"""In-step phase timeline of the fused LeNet step (one MI355X).

The PROF instantiations of the LeNet kernels record s_memrealtime (100 MHz, chip-global) per block at
phase boundaries (csrc/kernels/lenet.hip PMARK).  This captures a 1-step hipGraph with profiling on,
replays it, and prints for every kernel of the last replayed step: start / end relative to the step's
first block, block-start skew, and the median time from a block's start to each of its phase marks
(per role for the multi-role kernels).  Usage: python tools/lenet_phases.py [--steps-graph 1] [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_example_amd.data import synthetic_mnist  # noqa: E402
from pytorch_distributed_example_amd.engine import LeNetTrainStep  # noqa: E402
from pytorch_distributed_example_amd.models import build_net  # noqa: E402

NAMES = ["conv_fwd", "fc1_fwd", "head", "fc_bwd", "conv_bwd", "adam"]
ROLES = {3: {1: "B", 2: "C", 3: "A"}, 4: {1: "W", 2: "D", 3: "meter"}}


def analyse(buf):
    """buf: [6][4096][8] int64 -> dict of per-kernel stats (us)."""
    out = {}
    starts = {}
    for k, name in enumerate(NAMES):
        b = buf[k]
        live = b[:, 0] > 0
        if not live.any():
            continue
        starts[k] = b[live, 0].min()
    t0 = min(starts.values())
    tick = 0.01   # us per s_memrealtime tick
    for k, name in enumerate(NAMES):
        if k not in starts:
            continue
        b = buf[k]
        live = b[:, 0] > 0
        rows = b[live]
        st = rows[:, 0]
        ends = rows[:, 1:8].max(axis=1) if k == 0 else (rows[:, 1:7].max(axis=1) if k == 4 else rows[:, 1])
        rec = {"start": round((st.min() - t0) * tick, 2), "end": round((ends.max() - t0) * tick, 2),
               "blocks": int(live.sum()),
               "block_start_p50": round((np.median(st) - st.min()) * tick, 2),
               "block_start_max": round((st.max() - st.min()) * tick, 2),
               "block_dur_p50": round(float(np.median(ends - st)) * tick, 2),
               "block_dur_max": round(float((ends - st).max()) * tick, 2)}
        if k == 5:      # optimizer: which block ranges are slow (fold / pack ranges are contiguous)
            d = (ends - st) * tick
            idx = np.nonzero(live)[0]
            edges = np.linspace(0, idx.max() + 1, 17).astype(int)
            rec["dur_by_block_range"] = {f"{edges[i]}-{edges[i + 1]}": [
                round(float(np.median(d[(idx >= edges[i]) & (idx < edges[i + 1])])), 2),
                round(float(d[(idx >= edges[i]) & (idx < edges[i + 1])].max()), 2)]
                for i in range(16) if ((idx >= edges[i]) & (idx < edges[i + 1])).any()}
        if k == 0:
            rec["phases_p50"] = [round(float(np.median(rows[:, p] - st)) * tick, 2) for p in range(1, 8)
                                 if (rows[:, p] > 0).all()]
            idx = np.nonzero(live)[0]
            half = (idx.max() + 1) // 2       # 2-D grid (B, 2) flattened: [0, B) co-half / block column 0
            for c, sel in (("ct0", idx < half), ("ct1", idx >= half)):
                r = rows[sel]
                if len(r):
                    rec[f"phases_p50_{c}"] = [round(float(np.median(r[:, p] - r[:, 0])) * tick, 2)
                                              for p in range(1, 8) if (r[:, p] > 0).all()]
                    rec[f"end_max_{c}"] = round((r[:, 1:8].max(axis=1).max() - t0) * tick, 2)
        if k in ROLES:
            roles = {}
            for rid, rname in ROLES[k].items():
                sel = rows[:, 7] == rid
                if not sel.any():
                    continue
                r = rows[sel]
                nph = 7 if k == 4 else 2
                ph = []
                for p in range(1, nph):
                    v = r[:, p]
                    ok = v > 0
                    ph.append(round(float(np.median(v[ok] - r[ok, 0])) * tick, 2) if ok.any() else None)
                e = r[:, 1:7].max(axis=1) if k == 4 else r[:, 1]
                roles[rname] = {"n": int(sel.sum()), "start_p50": round((np.median(r[:, 0]) - t0) * tick, 2),
                                "start_max": round((r[:, 0].max() - t0) * tick, 2),
                                "end_max": round((e.max() - t0) * tick, 2), "phases_p50": ph}
            rec["roles"] = roles
        out[name] = rec
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--json", default=None)
    ap.add_argument("--bwd-dbg", type=int, default=0, help="ablation: 1 = conv_bwd2 without W, 2 = without D")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    net = build_net(seed=0, device=dev)
    eng = LeNetTrainStep(net, batch_size=a.B)
    eng.bwd_dbg = a.bwd_dbg
    ds = synthetic_mnist(60000, device=dev)
    eng.bind_dataset(ds.images, ds.labels)
    eng.set_epoch_indices(torch.randperm(60000, device=dev).to(torch.int32)[: (60000 // a.B) * a.B])
    for _ in range(20):
        eng.step()
    torch.cuda.synchronize()
    buf = torch.zeros(6 * 4096 * 8, dtype=torch.int64, device=dev)
    eng.K.lenet_set_prof(buf)
    g = eng.capture(steps=2)
    eng.K.lenet_set_prof(None)
    results = []
    for _ in range(a.reps):
        for _ in range(10):
            g.replay()
        buf.zero_()
        g.replay()
        torch.cuda.synchronize()
        results.append(analyse(buf.view(6, 4096, 8).cpu().numpy()))
    # median over reps of scalar fields
    med = {}
    for name in results[0]:
        r0 = results[0][name]
        m = {}
        for key, v in r0.items():
            if isinstance(v, (int, float)):
                m[key] = float(np.median([r[name][key] for r in results]))
            else:
                m[key] = v
        med[name] = m
    for name, r in med.items():
        print(name, json.dumps(r))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"median": med, "reps": results}, f, indent=1)


if __name__ == "__main__":
    main()
