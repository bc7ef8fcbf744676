#!/usr/bin/env python3
"""Store-ordering diagnostic for the persistent GEMMs (cfg 19 = k_gemm8pp, cfg 20 = k_gemm8pc).

Modes (GemmArgs::dbg bits 8-9, csrc/kernels/gemm.hip k_gemm8pp header):
  0  production: round 5's order (next tile's prologue, then this tile's stores), every wait vmcnt(VMW)
  1  round 5: the first K-tile waits vmcnt(VMW + NSTORE), counting the younger stores as still in flight
  2  construction (cfg 19, bf16 epilogue): round 5's waits, the real stores drained BEFORE the prologue and
     NSTORE decoy stores into an L2-resident 128 KB scratch where round 5 issued the real ones -- if a
     store can retire before an older load, the allowance lets phases read LDS slots that have not landed
  3  epilogue math under the prologue, vmcnt(0), then the stores (first K-tile waits skipped)

Part 1 (correctness): every mode x (fprop, dgrad, GELU forms) x shapes, R repeats, bit-compared against
cfg 18 (the one-shot 8-phase kernel: same per-accumulator k order).  Part 2 (timing): the GPT-2 shapes
per mode, graph-free CUDA-event timing.  Output: JSON lines."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributed_example_amd._ext import kernels  # noqa: E402
from pytorch_distributed_example_amd.ops import gemm as G  # noqa: E402


def bf(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to("cuda", torch.bfloat16)


def set_mode(m):
    kernels().gemm_set_dbg(m << 8)


_SCR = {}


def scratch(n):
    """decoy target for mode 2: the binding wants C2 as large as C; the kernel stores into its first 128 KB"""
    s = _SCR.get("s")
    if s is None or s.numel() < n:
        s = _SCR["s"] = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
    return s[:n]


def fprop_c2(x, w, b, c):
    """plain fprop with C2 = the decoy scratch (read only by mode 2)"""
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    kernels().gemm_bf16(x, w, y, 0, 0, G.EPI_BF16, M, N, K, K, K, N, 1, c, C2=scratch(M * N), bias=b)
    return y


def dgrad_c2(dy, w, c):
    M, Nk = dy.shape
    Ko = w.shape[1]
    dx = torch.empty(M, Ko, device="cuda", dtype=torch.bfloat16)
    kernels().gemm_bf16(dy, w, dx, 0, 1, G.EPI_BF16, M, Ko, Nk, Nk, Ko, Ko, 1, c, C2=scratch(M * Ko))
    return dx


def forms(M, N, K):
    """(name, fn(cfg) -> tuple of outputs) for one shape"""
    x, w, b = bf(M, K, seed=50), bf(N, K, scale=0.03, seed=51), bf(N, seed=52)
    dy, w2 = bf(M, K, seed=53), bf(K, N, scale=0.03, seed=54)
    dg = bf(M, N, seed=55)
    return [
        ("fprop", lambda c: (fprop_c2(x, w, b, c),)),
        ("fprop_gelu", lambda c: G.fprop(x, w, b, gelu=True, cfg=c)),
        ("dgrad", lambda c: (dgrad_c2(dy, w2, c),)),
        ("dgrad_gelu", lambda c: (G.dgrad(dy, w2, dgelu=dg, cfg=c),)),
    ]


def correctness(shapes, modes, cfgs, reps):
    for (M, N, K) in shapes:
        for name, fn in forms(M, N, K):
            set_mode(0)
            ref = fn(18)
            for cfg in cfgs:
                if cfg == 20 and (K % 128 or name == "dgrad_gelu"):
                    continue                      # runs another cfg
                for m in modes:
                    if m == 2 and (cfg != 19 or name not in ("fprop", "dgrad")):
                        continue
                    set_mode(m)
                    bad_runs, worst, bad_rows = 0, 0, set()
                    for _ in range(reps):
                        out = fn(cfg)
                        torch.cuda.synchronize()
                        nb = sum(int((o != r).sum()) for o, r in zip(out, ref))
                        if nb:
                            bad_runs += 1
                            worst = max(worst, nb)
                            rows = (out[0] != ref[0]).any(1).nonzero().flatten()
                            bad_rows.update((rows // 256).tolist())
                    print(json.dumps({"part": "correctness", "M": M, "N": N, "K": K, "form": name, "cfg": cfg,
                                      "mode": m, "reps": reps, "mismatching_runs": bad_runs,
                                      "max_mismatching_elems": worst, "bad_row_tiles": sorted(bad_rows)[:12]}),
                          flush=True)
    set_mode(0)


def timing(modes, iters):
    T = 16384
    cases = [  # GPT-2 step GEMMs that cfg 19 / 20 serve (ops/gemm.py _CFG), + cfg 18 reference
        ("fprop_gelu c_fc", T, 3072, 768, "fprop_gelu"),
        ("fprop lm_head nt", T, 50304, 768, "fprop_nt"),
        ("dgrad c_fc", T, 768, 3072, "dgrad"),
        ("dgrad_gelu c_proj", T, 3072, 768, "dgrad_gelu"),
        ("dgrad lm_head", T, 768, 50304, "dgrad"),
    ]
    for label, M, N, K, kind in cases:
        x, w, b = bf(M, K, seed=1), bf(N, K, scale=0.03, seed=2), bf(N, seed=3)
        w2 = bf(K, N, scale=0.03, seed=4)
        dg = bf(M, N, seed=5)
        if kind == "fprop_gelu":
            fn = lambda c: G.fprop(x, w, b, gelu=True, cfg=c)  # noqa: E731
        elif kind == "fprop_nt":
            fn = lambda c: G.fprop(x, w, None, cfg=c, nt_out=(c == 19))  # noqa: E731
        elif kind == "dgrad":
            fn = lambda c: G.dgrad(x, w2, cfg=c)  # noqa: E731
        else:
            fn = lambda c: G.dgrad(x, w2, dgelu=dg, cfg=c)  # noqa: E731
        runs = [(18, 0)] + [(19, m) for m in modes if m != 2]
        if K % 128 == 0 and kind in ("dgrad", "fprop_gelu"):
            runs += [(20, m) for m in modes if m != 2]
        best = {}
        for _rnd in range(3):                      # interleaved rounds, best of 3 (clock / thermal drift)
            for cfg, m in runs:
                set_mode(m)
                for _ in range(3):
                    fn(cfg)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    fn(cfg)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / iters
                best[(cfg, m)] = min(us, best.get((cfg, m), 1e30))
        for (cfg, m), us in best.items():
            tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
            print(json.dumps({"part": "timing", "case": label, "M": M, "N": N, "K": K, "cfg": cfg, "mode": m,
                              "us": round(us, 1), "tflops": round(tf, 1)}), flush=True)
        del x, w, b, w2, dg
        torch.cuda.empty_cache()
    set_mode(0)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--modes", default="0,1,2,3")
    ap.add_argument("--skip-timing", action="store_true")
    ap.add_argument("--skip-correctness", action="store_true")
    args = ap.parse_args()
    modes = [int(m) for m in args.modes.split(",")]
    if not args.skip_correctness:
        correctness([(9000, 3072, 768), (16384, 2304, 768), (4100, 776, 1536), (20000, 2056, 128)], modes,
                    [19, 20], args.reps)
    if not args.skip_timing:
        timing(modes, args.iters)
