"""Which part of bench.py's pre-window sequence makes its 20-step window slower than a plain
window right after warm-up: variants of the warm-up / meter reset / GC before the GPU-event-clocked
20-step replay, interleaved, each measured several times in one process."""
import gc
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
eng.prime_graphs((1, 5, 20), replays=3)


def window():
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    eng.replay(steps=20)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / 20


def variant(name):
    if name == "w1x5":
        for _ in range(5):
            eng.replay(steps=1)
    elif name == "w5":
        eng.replay(steps=5)
    elif name == "w5_reset":
        eng.replay(steps=5)
        eng.reset_meters()
    elif name == "w5_reset_gcoff":
        gc.collect()
        gc.disable()
        eng.replay(steps=5)
        eng.reset_meters()
    elif name == "w5_sync2":
        eng.replay(steps=5)
        eng.reset_meters()
        torch.cuda.synchronize()
    elif name == "w20":
        eng.replay(steps=20)
    torch.cuda.synchronize()
    if name == "w5_sync2":
        torch.cuda.synchronize()
    r = window()
    gc.enable()
    return r


names = ["w1x5", "w5", "w5_reset", "w5_reset_gcoff", "w5_sync2", "w20"]
res = {n: [] for n in names}
for rep in range(6):
    for n in names:
        time.sleep(0.05)                      # a settled, idle GPU before each trial, as in a fresh bench
        res[n].append(round(variant(n), 2))
print(json.dumps({n: {"median": sorted(v)[len(v) // 2], "all": v} for n, v in res.items()}))
