"""Ablation of the own GEMM's v1 main loop (kernels().gemm_set_dbg): time a GEMM with the LDS-DMA
staging (1), the waits + barriers (2) and/or the LDS fragment reads (4) switched off (results are
wrong; only the time matters), to see which part of the pipeline bounds it."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_example_amd._ext import kernels  # noqa: E402
from pytorch_distributed_example_amd.ops import gemm as G  # noqa: E402
from gemm_own_bench import timeit  # noqa: E402

dev = torch.device("cuda", 0)
r = lambda *s: (torch.randn(*s, device=dev) * 0.05).to(torch.bfloat16)
T = 16384
cases = {
    "c_fc.dgrad/cfg0": (lambda cfg: (lambda dy=r(T, 3072), w=r(3072, 768): lambda: G.dgrad(dy, w, cfg=cfg))(), 0),
    "mlp_proj.fprop/cfg0": (lambda cfg: (lambda x=r(T, 3072), w=r(768, 3072): lambda: G.fprop(x, w, cfg=cfg))(), 0),
    "c_attn.fprop/cfg0": (lambda cfg: (lambda x=r(T, 768), w=r(2304, 768): lambda: G.fprop(x, w, cfg=cfg))(), 0),
    "lm_head.fprop/cfg3": (lambda cfg: (lambda x=r(T, 768), w=r(50304, 768): lambda: G.fprop(x, w, cfg=cfg))(), 3),
}
for name, (mk, cfg) in cases.items():
    fn = mk(cfg)
    res = {}
    for d in (0, 1, 2, 3, 4, 5, 6, 7):
        kernels().gemm_set_dbg(d)
        res[d] = round(timeit(fn, 10), 1)
    kernels().gemm_set_dbg(0)
    print(json.dumps({"gemm": name, "us_by_dbg": res}), flush=True)
