"""Where the 20-step driver window's extra GPU time comes from (vs the long-run step time):
GPU-event-clocked 20-step windows right after the bench's warm-up, back to back, after a long busy
period, after idle gaps, and with the first step of the window split off into its own graph."""
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
eng.prime_graphs((20, 1), replays=3)


def window(n=20, S=20):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n // S):
        eng.replay(steps=S)
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1e3 / n, 2)


res = {}
for _ in range(5):
    eng.replay(steps=1)
res["after_warmup"] = window()
res["back_to_back"] = [window() for _ in range(5)]
for _ in range(50):
    eng.replay(steps=20)
res["after_1000_busy_steps"] = window()
res["long_100x20"] = window(2000)
for gap in (0.0001, 0.001, 0.01, 0.1):
    torch.cuda.synchronize()
    time.sleep(gap)
    res[f"after_idle_{gap * 1e3:g}ms"] = window()
# per-step GPU time inside one 20-step window: events between 1-step replays (S=1)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
ev[0].record()
for i in range(20):
    eng.replay(steps=1)
    ev[i + 1].record()
torch.cuda.synchronize()
res["per_step_S1_us"] = [round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i in range(20)]
print(json.dumps(res))
