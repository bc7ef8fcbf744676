#!/usr/bin/env python3
"""Causal flash-attention kernels (csrc/kernels/attention.hip) at the GPT-2 small shape
(B=16, T=1024, H=12, D=64): time per call and achieved TFLOP/s (causal FLOPs).

usage: python tools/attn_bench.py [--iters 20]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_distributed_example_amd._ext import kernels


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--variants", default="0", help="attention variant bits (pde_attn_set_variant), comma list")
    a = ap.parse_args()
    K = kernels()
    B, T, H, D = a.B, a.T, a.H, 64
    C = H * D
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3 * C, device="cuda").to(torch.bfloat16)
    q, k, v = qkv[:, :, :C], qkv[:, :, C:2 * C], qkv[:, :, 2 * C:]
    o = torch.empty(B, T, C, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device="cuda")
    do = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = dqkv[:, :, :C], dqkv[:, :, C:2 * C], dqkv[:, :, 2 * C:]
    Dd = torch.empty(B * H * T, device="cuda")
    scale = 1.0 / math.sqrt(D)
    fwd_flops = 4.0 * B * H * T * T * D / 2          # QK^T + PV, causal half
    for var in [int(x) for x in a.variants.split(",")]:
        K.attn_set_variant(var)
        t_f = timeit(lambda: K.attn_fwd(q, k, v, o, lse, H, scale), a.iters)
        t_b = timeit(lambda: K.attn_bwd(q, k, v, o, do, lse, Dd, dq, dk, dv, H, scale), a.iters)
        print(json.dumps({"variant": var, "shape": [B, T, H, D], "fwd_us": round(t_f, 1),
                          "fwd_tflops": round(fwd_flops / t_f / 1e6, 1), "bwd_us": round(t_b, 1),
                          "bwd_tflops": round(2.5 * fwd_flops / t_b / 1e6, 1)}), flush=True)
    K.attn_set_variant(5)


if __name__ == "__main__":
    main()
