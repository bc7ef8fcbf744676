"""Fixed per-window overhead of the headline timing (graph launch + final synchronize) on one
MI355X: wall time of replaying S-step graphs of the LeNet step, from an idle GPU, vs S."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_example_amd.data import synthetic_mnist  # noqa: E402
from pytorch_distributed_example_amd.engine import LeNetTrainStep  # noqa: E402
from pytorch_distributed_example_amd.models import build_net  # noqa: E402

dev = torch.device("cuda", 0)
net = build_net(seed=0, device=dev)
eng = LeNetTrainStep(net, batch_size=128)
ds = synthetic_mnist(60000, device=dev)
eng.bind_dataset(ds.images, ds.labels)
eng.set_epoch_indices(torch.randperm(60000, device=dev).to(torch.int32)[:59904])
for _ in range(20):
    eng.step()
torch.cuda.synchronize()
res = {}
# sync alone and a trivial kernel
t = []
for _ in range(20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    t.append(time.perf_counter() - t0)
res["sync_only_us"] = round(1e6 * sorted(t)[len(t) // 2], 1)
x = torch.zeros(1, device=dev)
t = []
for _ in range(20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x.add_(1)
    torch.cuda.synchronize()
    t.append(time.perf_counter() - t0)
res["tiny_kernel_us"] = round(1e6 * sorted(t)[len(t) // 2], 1)
for S in (1, 2, 10, 20, 40, 100):
    eng.graphs.clear()
    eng.capture(steps=S)
    eng.capture(steps=S)        # both parities
    for _ in range(3):
        eng.replay(steps=S)
    ts = []
    for _ in range(9):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.replay(steps=S)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    med = sorted(ts)[len(ts) // 2]
    res[f"S{S}_us"] = round(1e6 * med, 1)
    res[f"S{S}_us_per_step"] = round(1e6 * med / S, 2)
# the bench's exact window: idle gap (host work) before the timed replay
for gap_ms in (0.0, 0.2, 1.0, 10.0):
    ts = []
    for _ in range(9):
        torch.cuda.synchronize()
        if gap_ms:
            time.sleep(gap_ms / 1e3)
        t0 = time.perf_counter()
        eng.replay(steps=100)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res[f"S100_after_idle_{gap_ms}ms_us_per_step"] = round(1e6 * sorted(ts)[4] / 100, 2)
for gap_ms in (0.0, 1.0, 10.0):
    ts = []
    eng.graphs.clear()
    eng.capture(steps=20)
    eng.capture(steps=20)
    eng.replay(steps=20)
    eng.replay(steps=20)
    for _ in range(9):
        torch.cuda.synchronize()
        if gap_ms:
            time.sleep(gap_ms / 1e3)
        t0 = time.perf_counter()
        eng.replay(steps=20)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res[f"S20_after_idle_{gap_ms}ms_us_per_step"] = round(1e6 * sorted(ts)[4] / 20, 2)
print(json.dumps(res))
