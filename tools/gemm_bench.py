#!/usr/bin/env python3
"""Time the GPT-2 small GEMM shapes (bf16, 16x1024 tokens) on the library path and with split-K
for the long-K weight-gradient products; prints TFLOP/s per variant (JSON lines)."""
import json
import time

import torch

N = 16384
SHAPES = {"c_attn": (768, 2304), "attn.c_proj": (768, 768), "c_fc": (768, 3072), "mlp.c_proj": (3072, 768),
          "lm_head": (768, 50304)}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    dev = "cuda"
    torch.manual_seed(0)
    for name, (fin, fout) in SHAPES.items():
        x = torch.randn(N, fin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(fout, fin, device=dev, dtype=torch.bfloat16)
        b = torch.randn(fout, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(N, fout, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * N * fin * fout
        res = {"gemm": name, "M_N_K": [N, fout, fin]}
        res["fwd_linear"] = fl / timeit(lambda: torch.nn.functional.linear(x, w, b)) / 1e12
        res["dgrad_mm"] = fl / timeit(lambda: torch.matmul(dy, w)) / 1e12
        res["wgrad_mm"] = fl / timeit(lambda: torch.matmul(dy.t(), x)) / 1e12
        for S in (2, 4, 8):
            def splitk(S=S):
                p = torch.bmm(dy.view(S, N // S, fout).transpose(1, 2), x.view(S, N // S, fin))
                return p.sum(0)
            res[f"wgrad_splitk{S}"] = fl / timeit(splitk) / 1e12
        res["bias_grad_sum"] = timeit(lambda: dy.sum(0)) * 1e6
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
