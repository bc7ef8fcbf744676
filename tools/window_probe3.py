"""Fixed cost of a timed window of the toy-CNN step: host-clocked (sync, replay n steps, sync) and
GPU-event-clocked windows for n = 1..100 steps, the host time of the replay call itself, and 20 steps
launched as 1x20 / 2x10 / 4x5 graphs.  Fit t(n) = a + b*n: b is the steady-state step, a the per-window
cost the driver's 20-step window pays once."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_example_amd.utils.hipsched import set_schedule  # noqa: E402

set_schedule(0)
from pytorch_distributed_example_amd.data import DistributedSampler, synthetic_mnist  # noqa: E402
from pytorch_distributed_example_amd.engine import LeNetTrainStep  # noqa: E402
from pytorch_distributed_example_amd.models import build_net  # noqa: E402

dev = torch.device("cuda", 0)
net = build_net(seed=0, device=dev)
eng = LeNetTrainStep(net, batch_size=128)
ds = synthetic_mnist(60000, seed=0, device=dev, kind="fashion")
eng.bind_dataset(ds.images, ds.labels)
idx = DistributedSampler(ds, num_replicas=1, rank=0, shuffle=True, seed=0).indices_tensor()
eng.set_epoch_indices(idx[: (idx.numel() // 128) * 128])
NS = (1, 2, 5, 10, 20, 40, 100)
eng.prime_graphs(NS, replays=2)


def host_window(parts):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for n in parts:
        eng.replay(steps=n)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t2 - t0) * 1e6, (t1 - t0) * 1e6


def event_window(n):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    eng.replay(steps=n)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3


res = {f"host{n}": [] for n in NS}
res.update({f"launch{n}": [] for n in NS})
res.update({f"event{n}": [] for n in NS})
splits = {"20=1x20": (20,), "20=2x10": (10, 10), "20=4x5": (5, 5, 5, 5), "20=20x1": (1,) * 20}
res.update({k: [] for k in splits})
for rep in range(7):
    for n in NS:
        time.sleep(0.02)
        h, l = host_window((n,))
        res[f"host{n}"].append(round(h, 1))
        res[f"launch{n}"].append(round(l, 1))
        time.sleep(0.02)
        res[f"event{n}"].append(round(event_window(n), 1))
    for k, parts in splits.items():
        time.sleep(0.02)
        res[k].append(round(host_window(parts)[0], 1))
med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
fit = {}
for kind in ("host", "event"):
    xs = list(NS)
    ys = [med[f"{kind}{n}"] for n in NS]
    mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    fit[kind] = {"a_us": round(my - b * mx, 1), "b_us_per_step": round(b, 2)}
print(json.dumps({"median_us": med, "fit": fit, "all": res}))
