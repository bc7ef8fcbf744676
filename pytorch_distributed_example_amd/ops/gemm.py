"""The framework's own bf16 MFMA GEMM (``csrc/kernels/gemm.hip``) for the GPT-2 projections and the
tied LM head -- the reference's ``nn.Linear`` op class (/root/reference/mnist/main.py:136-137) at
GPT-2 shapes, with the epilogues a library GEMM cannot fuse:

* ``fprop(x, w, bias, gelu)``   y = x w^T + b; with ``gelu`` the kernel writes gelu(pre) (the next
                                projection's input) AND gelu'(pre) (the backward's factor) in one
                                pass; the pre-activation itself is never stored.
* ``dgrad(dy, w, dgelu)``       dx = dy w; with ``dgelu`` the GELU backward is applied in the
                                epilogue (dx = (dy w) * gelu'(pre), one multiply).
* ``wgrad(dy, x, dw, db)``      dw = dy^T x (split-K over tokens, fp32 slabs, one reduction kernel
                                that also folds the bias gradient db = sum_tokens dy, computed by
                                the GEMM's own MFMAs against a ones fragment).

All operands stay in their natural row-major layouts (the kernel reads transposed operands with
``ds_read_b64_tr_b16``); GPU-only, bf16 in / bf16 out, fp32 accumulation.

Tile configurations (``gemm_tile(cfg)``): 0 = 256x192, 1 = 256x128, 2 = 128x128, 3 = 256x256,
4 = 128x128 at two blocks per CU; 5-8 = the same tiles (256x256, 256x192, 256x128, 128x128 x2)
on the v2 main loop (32-deep sub-stages, fragments of the next sub-stage read across the barrier);
9-13 = v1 tiles with the next stage's LDS-DMA spread over 2 or 4 k-steps; 14 / 15 = persistent 9 / 11
(one block per CU walking the tiles, each tile's output stores draining under the next tile's K loop;
fprop / dgrad only -- wgrad calls with these ids run 9 / 11); 16 / 17 = 256x192 / 256x256 on
v_mfma_f32_16x16x32_bf16 (every operand layout: fprop, dgrad, split-K wgrad); 18 = the 8-phase
256x256 loop (every layout); 19 = 18 in a persistent block per CU (fprop / dgrad; wgrad and other calls
run 18); 20 = 18 as one continuous K-tile stream per persistent block with a register epilogue (bias
fprop, plain dgrad, K % 128 == 0; other calls run 19); 21 = 20 at 256x192 (fprop; other calls run 16); 22 = 18 at 256x192 (fprop; other calls run 16).
``_CFG`` holds the per-shape choices measured on MI355X (``tools/gemm_own_bench.py`` ->
``profiles/r2_gemm/``); other shapes use the wave-quantisation heuristic of ``pick``.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch

from .._ext import kernels

EPI_BF16, EPI_GELU, EPI_GELU_BWD, EPI_SLAB = 0, 1, 2, 3
N_CU = 256
_TILES = {0: (256, 192), 1: (256, 128), 2: (128, 128), 3: (256, 256), 4: (128, 128),
          5: (256, 256), 6: (256, 192), 7: (256, 128), 8: (128, 128), 9: (256, 192), 10: (256, 192),
          11: (256, 256), 12: (256, 256), 13: (256, 128), 14: (256, 192), 15: (256, 256),
          16: (256, 192), 17: (256, 256), 18: (256, 256), 19: (256, 256), 20: (256, 256), 21: (256, 192), 22: (256, 192)}
# relative per-CU throughput of a full tile wave (bigger tiles re-read less through L2)
_TILE_EFF = {0: 1.0, 1: 0.93, 2: 0.8, 3: 1.0, 4: 0.85, 5: 0.9, 6: 0.9, 7: 0.85, 8: 0.8, 9: 1.0, 10: 1.0, 11: 1.0,
             12: 1.0, 13: 0.93, 14: 0.99, 15: 0.99, 16: 1.0, 17: 1.0, 18: 1.0, 19: 1.0, 20: 1.0, 21: 1.0, 22: 1.0}

# GPT-2-small GEMMs at 16384 tokens, measured on MI355X (tools/gemm_own_bench.py, profiles/r2_gemm/,
# profiles/r3_gemm/):
#   fprop / dgrad: (kind, N, K) -> (cfg, 1) for M >= 4096 rows
#   wgrad:         (kind, M, N) -> (cfg, splits at 16384 tokens; scaled with the token count)
_CFG: Dict[Tuple[str, int, int], Tuple[int, int]] = {
    # round 5 (profiles/r5_gemm/, profiles/r5_gpt2/): every GPT-2 GEMM on the framework's kernels, no
    # library fallback -- the 8-phase loop at 256x192 (cfg 22) for the N = 768 output projections (one
    # tile round on 256 CUs, on par with hipBLASLt), the 16x16x32 loop at 256x192 (cfg 16) for c_attn
    # (12 column tiles: 3 exact rounds), the persistent 8-phase loop
    # (cfg 19) for the GELU fprop, the GELU-backward dgrad and the LM head (whose fprop stores the 1.65 GB
    # of logits non-temporally: within 3 % of hipBLASLt, 12 % faster than plain stores)
    ("fprop", 2304, 768): (16, 1), ("fprop", 768, 768): (22, 1), ("fprop", 3072, 768): (19, 1),
    ("fprop", 768, 3072): (22, 1), ("fprop", 50304, 768): (19, 1),
    # dgrad: the persistent cfg 19 again for the GELU-backward and LM-head dgrads (round 6: its tile-
    # boundary waits no longer count stores as in flight, profiles/r6_gemm/; 90.5 vs 95.1 us and
    # 1021 vs 1140 us against cfg 18), cfg 18 for the plain mlp dgrad (74.3 vs 76.9 us)
    ("dgrad", 768, 2304): (9, 1), ("dgrad", 768, 768): (9, 1), ("dgrad", 768, 3072): (18, 1),
    ("dgrad", 3072, 768): (19, 1), ("dgrad", 768, 50304): (19, 1),
    # split counts that bring tiles x splits closest to the 256 CUs (profiles/r3_gemm/; 256x256 tiles
    # for cfg 18: 36 tiles x 7, 27 x 9)
    ("wgrad", 2304, 768): (18, 9), ("wgrad", 768, 768): (9, 16), ("wgrad", 3072, 768): (18, 7),
    ("wgrad", 768, 3072): (18, 7), ("wgrad", 50304, 768): (18, 1),
}


def _env_overrides() -> None:
    """PDE_GEMM_CFG="fprop:3072:768=15,wgrad:3072:768=9/5" replaces table entries (same-box A/B runs):
    kind:a:b as the table keys, cfg[/splits]."""
    import os
    spec = os.environ.get("PDE_GEMM_CFG", "").strip()
    for item in filter(None, (x.strip() for x in spec.split(","))):
        key, val = item.split("=")
        kind, a, b = key.split(":")
        cfg, _, sp = val.partition("/")
        _CFG[(kind, int(a), int(b))] = (int(cfg), int(sp) if sp else 1)


_env_overrides()


_SCRATCH: Dict[Tuple, torch.Tensor] = {}


def _scratch(device, n: int, tag: str) -> torch.Tensor:
    key = (device, tag)
    t = _SCRATCH.get(key)
    if t is None or t.numel() < n:
        t = torch.empty(max(n, 1), device=device, dtype=torch.float32)
        _SCRATCH[key] = t
    return t[:n]


def pick(kind: str, M: int, N: int, K: int) -> Tuple[int, int]:
    """(cfg, splits) for a GEMM: the measured table, else the config whose last wave of tiles
    wastes the least of the chip (tiles / (rounds * CUs) x tile efficiency); wgrad also picks a
    split-K factor that brings the tile count to >= 1 round with >= 1024-deep slices."""
    if kind == "wgrad":
        hit = _CFG.get((kind, M, N))
        if hit is not None and K >= 2048:
            return hit[0], max(1, min(hit[1], round(hit[1] * K / 16384)))
    else:
        hit = _CFG.get((kind, N, K))
        if hit is not None and M >= 4096:
            return hit
    best, best_s = None, -1.0
    for cfg, (bm, bn) in _TILES.items():
        tiles = math.ceil(M / bm) * math.ceil(N / bn)
        splits = 1
        if kind == "wgrad":
            while tiles * splits < N_CU and K // (64 * splits * 2) >= 16:
                splits *= 2
        tot = tiles * splits
        rounds = math.ceil(tot / N_CU)
        score = tot / (rounds * N_CU) * _TILE_EFF[cfg]
        if kind == "wgrad" and splits > 1:
            score *= 0.97                                # slab round trip + reduction
        if score > best_s + 1e-9:
            best, best_s = (cfg, splits), score
    return best


def _chk(t: torch.Tensor, name: str):
    if not (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous()):
        raise ValueError(f"gemm: {name} must be a contiguous bf16 GPU tensor")


def fprop(x2: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, gelu: bool = False,
          out: Optional[torch.Tensor] = None, cfg: Optional[int] = None, nt_out: bool = False):
    """x2 [M, K] . w[N, K]^T (+ bias) -> y [M, N]; with ``gelu`` returns (gelu(y), gelu'(y)).
    ``nt_out``: store y non-temporally (the persistent cfg 19 only; for outputs far larger than the
    caches, e.g. the LM-head logits)."""
    _chk(x2, "x")
    _chk(w, "w")
    M, K = x2.shape
    N = w.shape[0]
    c = pick("fprop", M, N, K)[0] if cfg is None else cfg
    y = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16) if out is None else out
    if gelu:
        dgelu = torch.empty_like(y)
        kernels().gemm_bf16(x2, w, y, 0, 0, EPI_GELU, M, N, K, K, K, N, 1, c, C2=dgelu, bias=bias)
        return y, dgelu
    kernels().gemm_bf16(x2, w, y, 0, 0, EPI_BF16, M, N, K, K, K, N, 1, c | (256 if nt_out else 0), bias=bias)
    return y


def dgrad(dy2: torch.Tensor, w: torch.Tensor, dgelu: Optional[torch.Tensor] = None, cfg: Optional[int] = None,
          scale: Optional[torch.Tensor] = None, splits: Optional[int] = None):
    """dy2 [M, N] . w [N, K] -> dx [M, K]; with ``dgelu`` ([M, K], gelu'(pre) from ``fprop(gelu=True)``)
    returns dx * dgelu; ``scale`` (a one-element fp32 device tensor, e.g. the loss gradient) multiplies
    the result in the epilogue.  ``splits`` > 1 (no ``dgelu``): split-K over the reduction into fp32 slabs
    folded by one reduction kernel -- for deep reductions onto too few output tiles to fill the chip (the
    LM head: 50304-deep onto 64 x 3 tiles of 256 x 256)."""
    _chk(dy2, "dy")
    _chk(w, "w")
    M, Nk = dy2.shape                  # reduction over the weight's rows
    Kout = w.shape[1]
    c0, s0 = pick("dgrad", M, Kout, Nk)
    c = c0 if cfg is None else cfg
    S = s0 if splits is None else splits
    S = kernels().gemm_splits(Nk, S) if dgelu is None else 1
    dx = torch.empty(M, Kout, device=dy2.device, dtype=torch.bfloat16)
    if S > 1:
        part = _scratch(dy2.device, S * M * Kout, "slab")
        kernels().gemm_bf16(dy2, w, part, 0, 1, EPI_SLAB, M, Kout, Nk, Nk, Kout, Kout, S, c)
        kernels().gemm_reduce(part, S, M, Kout, dx, None, None, scale)
        return dx
    if dgelu is not None:
        kernels().gemm_bf16(dy2, w, dx, 0, 1, EPI_GELU_BWD, M, Kout, Nk, Nk, Kout, Kout, 1, c, aux=dgelu)
    else:
        kernels().gemm_bf16(dy2, w, dx, 0, 1, EPI_BF16, M, Kout, Nk, Nk, Kout, Kout, 1, c, scale=scale)
    return dx


def wgrad(dy2: torch.Tensor, x2: torch.Tensor, dw: Optional[torch.Tensor] = None, db: Optional[torch.Tensor] = None,
          want_db: bool = False, cfg: Optional[int] = None, splits: Optional[int] = None,
          scale: Optional[torch.Tensor] = None):
    """dw [N, K] = dy2[T, N]^T . x2[T, K] (into ``dw`` when given); with ``want_db`` (or ``db``) also
    db [N] = column sums of dy2.  ``scale``: one-element fp32 device tensor multiplying dw (not db).
    Returns (dw, db or None)."""
    _chk(dy2, "dy")
    _chk(x2, "x")
    T, N = dy2.shape
    K = x2.shape[1]
    c0, s0 = pick("wgrad", N, K, T)
    c = c0 if cfg is None else cfg
    S = kernels().gemm_splits(T, s0 if splits is None else splits)
    if dw is None:
        dw = torch.empty(N, K, device=dy2.device, dtype=torch.bfloat16)
    want_db = want_db or db is not None
    if want_db and db is None:
        db = torch.empty(N, device=dy2.device, dtype=torch.bfloat16)
    cs = _scratch(dy2.device, S * N, "cs") if want_db else None
    if S == 1:
        kernels().gemm_bf16(dy2, x2, dw, 1, 1, EPI_BF16, N, K, T, N, K, K, 1, c, colsum=cs, scale=scale)
        if want_db:
            kernels().gemm_reduce(None, 1, N, K, None, cs, db)     # db only
        return dw, db
    part = _scratch(dy2.device, S * N * K, "slab")
    kernels().gemm_bf16(dy2, x2, part, 1, 1, EPI_SLAB, N, K, T, N, K, K, S, c, colsum=cs)
    kernels().gemm_reduce(part, S, N, K, dw, cs, db, scale)
    return dw, db

