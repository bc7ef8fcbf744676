"""Own bf16 MFMA GEMM (csrc/kernels/gemm.hip) vs the library GEMM (torch.matmul -> hipBLASLt) at
every GPT-2-small GEMM of one training step (B=16, T=1024 -> 16384 tokens), all tile configs and,
for wgrad, split-K factors.  One JSON line per GEMM: us and TFLOP/s of the library and of every
own candidate, and the best candidate (the table ``ops/gemm.py:_CFG`` is filled from these).

    python tools/gemm_own_bench.py [--tokens 16384] [--iters 20] [--only fprop,dgrad,wgrad]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_example_amd.ops import gemm as G  # noqa: E402

C, V = 768, 50304


def timeit(fn, iters, rounds=2):
    """us per call: the best of ``rounds`` timed runs of ``iters`` calls (the first config timed after a
    library call measured up to 12 % slow in a single run, profiles/r5_gemm/)."""
    best = float("inf")
    for _ in range(rounds):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="fprop,dgrad,wgrad")
    ap.add_argument("--out", default=None)
    ap.add_argument("--cfgs", default="9,11,14,15,16,17")
    a = ap.parse_args()
    T = a.tokens
    CFGS = [int(c) for c in a.cfgs.split(",")]
    dev = torch.device("cuda", 0)
    kinds = a.only.split(",")
    r = lambda *s: (torch.randn(*s, device=dev) * 0.05).to(torch.bfloat16)
    # (name, out, in, gelu-fused)
    layers = [("c_attn", 3 * C, C, False), ("attn_proj", C, C, False), ("c_fc", 4 * C, C, True),
              ("mlp_proj", C, 4 * C, False), ("lm_head", V, C, False)]
    lines = []
    for name, out, fin, gelu in layers:
        x, w, b = r(T, fin), r(out, fin), r(out)
        dy = r(T, out)
        flops = 2.0 * T * out * fin
        if "fprop" in kinds:
            lib = timeit(lambda: torch.nn.functional.linear(x, w, None if name == "lm_head" else b), a.iters)
            res = {}
            for cfg in CFGS:
                res[cfg] = timeit(lambda: G.fprop(x, w, None if name == "lm_head" else b, gelu=gelu, cfg=cfg), a.iters)
            best = min(res, key=res.get)
            lines.append({"gemm": f"{name}.fprop", "M": T, "N": out, "K": fin, "epilogue": "bias+gelu" if gelu else "bias",
                          "lib_us": round(lib, 1), "lib_tflops": round(flops / lib / 1e6, 1),
                          "own_us": {c: round(v, 1) for c, v in res.items()}, "best": best,
                          "own_tflops": round(flops / res[best] / 1e6, 1), "pick": G.pick("fprop", T, out, fin)})
            print(json.dumps(lines[-1]), flush=True)
        if "dgrad" in kinds:
            # dx [T, fin] = dy [T, out] . w [out, fin]; GELU backward fused for mlp_proj's input (c_fc act)
            pre = r(T, fin) if name == "mlp_proj" else None
            lib = timeit(lambda: torch.matmul(dy, w), a.iters)
            res = {}
            for cfg in CFGS:
                res[cfg] = timeit(lambda: G.dgrad(dy, w, dgelu=pre, cfg=cfg, splits=1), a.iters)
            if pre is None and fin * T <= 768 * 16384 and out >= 3072:   # deep reductions onto few tiles
                for cfg in (18, 9, 16):
                    for s in (2, 3, 4, 6):
                        res[f"{cfg}/{s}"] = timeit(lambda: G.dgrad(dy, w, cfg=cfg, splits=s), a.iters)
            best = min(res, key=res.get)
            lines.append({"gemm": f"{name}.dgrad", "M": T, "N": fin, "K": out,
                          "epilogue": "gelu_bwd" if pre is not None else "none",
                          "lib_us": round(lib, 1), "lib_tflops": round(flops / lib / 1e6, 1),
                          "own_us": {c: round(v, 1) for c, v in res.items()}, "best": best,
                          "own_tflops": round(flops / res[best] / 1e6, 1), "pick": G.pick("dgrad", T, fin, out)})
            print(json.dumps(lines[-1]), flush=True)
        if "wgrad" in kinds:
            dw = torch.empty(out, fin, device=dev, dtype=torch.bfloat16)
            lib = timeit(lambda: torch.matmul(dy.t(), x, out=dw), a.iters)
            res = {}
            for cfg in [c for c in CFGS if c in (0, 3, 4, 6, 9, 10, 11, 12, 13, 16, 17, 18)]:
                for s in (1, 2, 4, 5, 6, 7, 8, 9, 12, 16, 20, 26):
                    if name == "lm_head" and s > 2:
                        continue
                    res[f"{cfg}/{s}"] = timeit(lambda: G.wgrad(dy, x, dw=dw, want_db=name != "lm_head", cfg=cfg,
                                                               splits=s), a.iters)
            best = min(res, key=res.get)
            lines.append({"gemm": f"{name}.wgrad", "M": out, "N": fin, "K": T,
                          "epilogue": "bias-grad" if name != "lm_head" else "none",
                          "lib_us": round(lib, 1), "lib_tflops": round(flops / lib / 1e6, 1),
                          "own_us": {c: round(v, 1) for c, v in res.items()}, "best": best,
                          "own_tflops": round(flops / res[best] / 1e6, 1), "pick": G.pick("wgrad", out, fin, T)})
            print(json.dumps(lines[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for l in lines:
                f.write(json.dumps(l) + "\n")


if __name__ == "__main__":
    main()
