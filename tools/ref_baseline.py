"""Same-hardware baseline: the reference's training loop on stock PyTorch-ROCm ops.

Mirrors the per-step work of /root/reference/mnist/main.py:78-101 (Trainer.train) with
the model of mnist/main.py:130-147 and the DP sync of mnist/main.py:122-127, but on
synthetic MNIST-shaped data (no torchvision, no network).  Used ONLY to establish the
number our framework must beat on MI355X; nothing here is part of the framework.

Modes:
  faithful : .item() syncs per step as in the reference (loss.item(), accuracy .item())
  nosync   : same math, metric syncs removed (stock torch upper bound)
"""
import argparse, json, os, time
import torch
import torch.nn as nn
import torch.nn.functional as F


class StockNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 20, 5, 1)
        self.conv2 = nn.Conv2d(20, 50, 5, 1)
        self.fc1 = nn.Linear(800, 500)
        self.fc2 = nn.Linear(500, 10)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.conv1(x)), 2, 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2, 2)
        x = F.relu(self.fc1(x.view(-1, 800)))
        return F.log_softmax(self.fc2(x), dim=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--mode", default="faithful")
    ap.add_argument("--dist", action="store_true", help="RCCL per-param all_reduce (world from env)")
    a = ap.parse_args()
    rank = int(os.environ.get("RANK", 0)); world = int(os.environ.get("WORLD_SIZE", 1))
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    torch.cuda.set_device(dev)
    if a.dist:
        import torch.distributed as dist
        dist.init_process_group("nccl", rank=rank, world_size=world)
    net = StockNet().to(dev)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    n = 60000
    data = torch.randn(n, 1, 28, 28, device="cpu")
    labels = torch.randint(0, 10, (n,))
    perm = torch.randperm(n)

    def step(i):
        idx = perm[(i * a.batch) % (n - a.batch):][: a.batch]
        x = data[idx].to(dev, non_blocking=False); y = labels[idx].to(dev)
        out = net(x); loss = F.cross_entropy(out, y)
        opt.zero_grad(); loss.backward()
        if a.dist:
            for p in net.parameters():
                dist.all_reduce(p.grad.data, op=dist.ReduceOp.SUM); p.grad.data /= float(world)
        opt.step()
        if a.mode == "faithful":
            loss.item(); out.argmax(dim=1).eq(y).sum().item()

    for i in range(a.warmup): step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps): step(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ips = a.steps * a.batch * world / dt
    if rank == 0:
        print(json.dumps({"baseline": "stock-torch reference loop", "mode": a.mode, "dist": a.dist,
                          "world": world, "images_per_s": round(ips, 1),
                          "ms_per_step": round(dt / a.steps * 1e3, 4), "batch": a.batch}))


if __name__ == "__main__":
    main()
