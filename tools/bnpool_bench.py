#!/usr/bin/env python3
"""Time the fused stem-tail forward (BN finalize + apply + ReLU + 3x3/2 max-pool, k_bnpool_fwd*) at the
ResNet-18 geometry (B x 64 x 112 x 112, channels-last bf16) for each PDE_BNPOOL_FWD variant (pooled
cells per thread: 1, 2, 4), interleaved rounds in one process.

usage: python tools/bnpool_bench.py [--batch 256] [--iters 50] [--rounds 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_distributed_example_amd.models.resnet import BN
from pytorch_distributed_example_amd.ops.resnet import bn_relu_maxpool


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    C, H = 64, 112
    y = torch.randn(args.batch, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, C)
    stats = (torch.cat([yf.sum(0), (yf * yf).sum(0)]).contiguous(), 1)
    del yf
    bn = BN(C).cuda().to(torch.bfloat16)
    res = {v: [] for v in ("1", "2", "4")}
    with torch.no_grad():
        for _ in range(args.rounds):
            for v in res:
                os.environ["PDE_BNPOOL_FWD"] = v
                bn_relu_maxpool(y, stats, bn)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    bn_relu_maxpool(y, stats, bn)
                e.record()
                torch.cuda.synchronize()
                res[v].append(s.elapsed_time(e) / args.iters * 1e3)
    for v, ts in res.items():
        print(json.dumps({"variant": int(v), "us": round(min(ts), 1), "all": [round(t, 1) for t in ts]}))


if __name__ == "__main__":
    main()
