#!/usr/bin/env python3
"""Stress check of the persistent GEMM (cfg 19) FPROP paths (the dgrad paths are disabled,
profiles/r5_gemm/rejected_cfg19_dgrad/): 30 repeats per shape of plain / GELU fprop against cfg 18,
ragged and full shapes, incl. the GPT-2 c_fc (GELU) and LM-head (non-temporal) shapes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_distributed_example_amd.ops import gemm as G


def bf(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to("cuda", torch.bfloat16)


REPS = 30
for (M, N, K, gelu) in [(9000, 3072, 768, False), (9000, 3072, 768, True), (16384, 3072, 768, True),
                        (16384, 50304, 768, False), (4100, 776, 1536, False)]:
    x, w, b = bf(M, K, seed=50), bf(N, K, scale=0.03, seed=51), bf(N, seed=52)
    ref = G.fprop(x, w, b, gelu=gelu, cfg=18)
    bad = 0
    for _ in range(REPS):
        o = G.fprop(x, w, b, gelu=gelu, cfg=19)
        ok = (torch.equal(o[0], ref[0]) and torch.equal(o[1], ref[1])) if gelu else torch.equal(o, ref)
        bad += not ok
    torch.cuda.synchronize()
    print(f"fprop M={M} N={N} K={K} gelu={gelu}: mismatching repeats {bad} / {REPS}", flush=True)
