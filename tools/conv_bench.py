#!/usr/bin/env python3
"""Per-layer timing of the implicit-GEMM MFMA convolutions (conv.hip) vs MIOpen (F.conv2d) on every
ResNet-18 conv geometry at batch 256, channels-last bf16.  Interleaved rounds in one process.

usage: python tools/conv_bench.py [--batch 256] [--iters 20]
       python tools/conv_bench.py --wgrad-sweep 0.5 1 2 3   (wgrad only: split count x factor, per depth)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from pytorch_distributed_example_amd._ext import kernels

# name, Cin, H, Cout, k, stride, pad, count in the network
LAYERS = [
    ("l1.conv", 64, 56, 64, 3, 1, 1, 4),
    ("l2.0.conv1", 64, 56, 128, 3, 2, 1, 1),
    ("l2.ds", 64, 56, 128, 1, 2, 0, 1),
    ("l2.conv", 128, 28, 128, 3, 1, 1, 3),
    ("l3.0.conv1", 128, 28, 256, 3, 2, 1, 1),
    ("l3.ds", 128, 28, 256, 1, 2, 0, 1),
    ("l3.conv", 256, 14, 256, 3, 1, 1, 3),
    ("l4.0.conv1", 256, 14, 512, 3, 2, 1, 1),
    ("l4.ds", 256, 14, 512, 1, 2, 0, 1),
    ("l4.conv", 512, 7, 512, 3, 1, 1, 3),
]


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--stages", type=int, nargs="+", default=[3, 2], help="LDS pipeline depths to time")
    ap.add_argument("--wgrad-sweep", type=float, nargs="+", default=None,
                    help="wgrad only: time split counts default x these factors at every depth")
    ap.add_argument("--wgrad-blocks", type=float, nargs="+", default=None,
                    help="with --wgrad-sweep: split counts floor(k * 512 / tiles) for these k instead")
    args = ap.parse_args()
    if args.wgrad_sweep or args.wgrad_blocks:
        return wgrad_sweep(args)
    K = kernels()
    dev = "cuda"
    B = args.batch
    tot = {"ours": 0.0, "miopen": 0.0}
    for name, C, H, N, k, s, p, cnt in LAYERS:
        torch.manual_seed(0)
        x = torch.randn(B, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(N, C, k, k, device=dev) / (C * k * k) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        OH = (H + 2 * p - k) // s + 1
        y = torch.empty(B, N, OH, OH, device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        wt = torch.empty(w.numel(), device=dev, dtype=torch.bfloat16)
        splits = K.conv_wgrad_splits(x, w, s, p)
        part = torch.empty(splits * w.numel(), device=dev)
        flops = 2.0 * B * OH * OH * N * C * k * k
        xr = x.detach().requires_grad_()
        wr = w.detach().requires_grad_()
        res = {}
        for rnd in range(2):
            for nst in args.stages:
                K.conv_set_stages(nst)
                sfx = "" if nst == args.stages[0] else f"_nst{nst}"
                res["fprop" + sfx] = timeit(lambda: K.conv_fprop(x, w, y, None, s, p), args.iters)
                res["dgrad" + sfx] = timeit(lambda: K.conv_dgrad(dy, w, wt, dx, s, p), args.iters)
                res["wgrad" + sfx] = timeit(lambda: K.conv_wgrad(dy, x, w, part, splits, dw, s, p), args.iters)
            K.conv_set_stages(args.stages[0])
            res["mi_fprop"] = timeit(lambda: F.conv2d(x, w, None, s, p), args.iters)
            res["mi_dgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
                dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False]), args.iters)
            res["mi_wgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
                dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False]), args.iters)
        out = {"layer": name, "count": cnt, "gflop": round(flops / 1e9, 2), "splits": splits}
        for kk, v in res.items():
            out[kk + "_us"] = round(v, 1)
            out[kk + "_tflops"] = round(flops / v / 1e6, 1)
        ours = res["fprop"] + res["dgrad"] + res["wgrad"]
        mi = res["mi_fprop"] + res["mi_dgrad"] + res["mi_wgrad"]
        tot["ours"] += cnt * ours
        tot["miopen"] += cnt * mi
        print(json.dumps(out), flush=True)
    print(json.dumps({"total_us_per_step_ours": round(tot["ours"], 1),
                      "total_us_per_step_miopen": round(tot["miopen"], 1)}), flush=True)


def wgrad_sweep(args):
    K = kernels()
    dev = "cuda"
    B = args.batch
    for name, C, H, N, k, s, p, cnt in LAYERS:
        torch.manual_seed(0)
        x = torch.randn(B, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(N, C, k, k, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        OH = (H + 2 * p - k) // s + 1
        dy = torch.randn(B, N, OH, OH, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dw = torch.empty_like(w)
        s0 = K.conv_wgrad_splits(x, w, s, p)
        flops = 2.0 * B * OH * OH * N * C * k * k
        ref = None
        BM = 128 if N % 128 == 0 else 64
        tiles = (N // BM) * ((k * k * C + 127) // 128)
        if args.wgrad_blocks:
            cands = sorted({s0} | {max(1, int(f * 512) // tiles) for f in args.wgrad_blocks})
        else:
            cands = [max(1, int(round(s0 * f))) for f in args.wgrad_sweep]
        for sp in cands:
            part = torch.empty(sp * w.numel(), device=dev)
            for nst in args.stages:
                K.conv_set_stages(nst)
                us = min(timeit(lambda: K.conv_wgrad(dy, x, w, part, sp, dw, s, p), args.iters) for _ in range(2))
                if ref is None:
                    ref = dw.float().clone()
                err = ((dw.float() - ref).norm() / ref.norm()).item()
                print(json.dumps({"layer": name, "count": cnt, "splits": sp, "default_splits": s0, "nst": nst,
                                  "blocks": sp * tiles,
                                  "us": round(us, 1), "tflops": round(flops / us / 1e6, 1), "rel_vs_first": err}),
                      flush=True)
        K.conv_set_stages(2)


if __name__ == "__main__":
    main()
