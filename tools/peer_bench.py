"""Microbenchmark: all-reduce routes at the toy CNN's bucket sizes (us per call, max over ranks).

  python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 tools/peer_bench.py [--shared-gpu]

On an 8-GPU node this compares RCCL with the xGMI peer kernels (one-shot / two-shot) exactly as the
engine's start-up tuning does.  With --shared-gpu every rank uses cuda:0 (1-GPU rehearsal: only the
kernels' fixed costs are meaningful, the transport is local HBM).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_example_amd import dist  # noqa: E402
from pytorch_distributed_example_amd.dist.peer import PeerAllReduce, tune_routes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shared-gpu", action="store_true")
    ap.add_argument("--sizes", default="25360,405720,431080,1048576,4194304")
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = 0 if a.shared_gpu else int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("gloo" if a.shared_gpu else "nccl", init_method="env://", rank=rank, world_size=world)
    g = dist.get_default_group()
    sizes = [int(x) for x in a.sizes.split(",")]
    peer = PeerAllReduce(g, dev, max(sizes) * 4)
    rccl_fn = None
    if g.rccl is not None:
        def rccl_fn(t):
            g.rccl.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), 0, 0, torch.cuda.current_stream().cuda_stream)
    routes, times = tune_routes(g, peer if peer.ok else None, rccl_fn, sizes, dev, iters=a.iters)
    if rank == 0:
        print(json.dumps({"world": world, "shared_gpu": a.shared_gpu, "peer_ok": peer.ok, "peer_reason": peer.reason,
                          "routes": {str(k): v for k, v in routes.items()},
                          "us_per_call": {str(k): v for k, v in times.items()}}), flush=True)
    peer.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
