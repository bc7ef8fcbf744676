"""GPT-2 (124M, "small") in bf16 over the framework's transformer ops.

Driver-added config of BASELINE.json ("GPT-2-small transformer DDP 8xMI355X: large grad buckets,
MFMA GEMM + fused Adam"); the reference itself has no transformer (survey §2.5).  Architecture =
GPT-2 small: 12 layers, 12 heads x 64, d_model 768, context 1024, vocab 50257 padded to 50304 (a
multiple of 128, for GEMM tiling), pre-LayerNorm blocks, tanh-GELU MLP (4x), tied token embedding /
LM head, learned positions.  Parameter names follow the common GPT-2 checkpoint layout
(``transformer.wte.weight``, ``transformer.h.{i}.attn.c_attn.weight`` [3C, C], ...); weights are
stored bf16 (the fused AdamW keeps the fp32 master copy).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as tnn

from ..ops import transformer as T


@dataclass
class GPTConfig:
    block_size: int = 1024
    vocab_size: int = 50257
    padded_vocab: int = 50304
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    ln_eps: float = 1e-5


class _LN(tnn.Module):
    def __init__(self, C, eps):
        super().__init__()
        self.weight = tnn.Parameter(torch.ones(C))
        self.bias = tnn.Parameter(torch.zeros(C))
        self.eps = eps

    def forward(self, x):
        return T.layer_norm(x, self.weight, self.bias, self.eps)


class _Linear(tnn.Module):
    def __init__(self, fin, fout, std):
        super().__init__()
        self.weight = tnn.Parameter(torch.empty(fout, fin).normal_(0.0, std))
        self.bias = tnn.Parameter(torch.zeros(fout))

    def forward(self, x):
        return T.linear(x, self.weight, self.bias)


class _Attn(tnn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        C = cfg.n_embd
        self.n_head = cfg.n_head
        self.c_attn = _Linear(C, 3 * C, 0.02)
        self.c_proj = _Linear(C, C, 0.02 / math.sqrt(2 * cfg.n_layer))

    def forward(self, x):
        return self.c_proj(T.causal_attention(self.c_attn(x), self.n_head))


class _MLP(tnn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        C = cfg.n_embd
        self.c_fc = _Linear(C, 4 * C, 0.02)
        self.c_proj = _Linear(4 * C, C, 0.02 / math.sqrt(2 * cfg.n_layer))

    def forward(self, x):
        return T.mlp(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias)


class Block(tnn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.ln_1 = _LN(cfg.n_embd, cfg.ln_eps)
        self.attn = _Attn(cfg)
        self.ln_2 = _LN(cfg.n_embd, cfg.ln_eps)
        self.mlp = _MLP(cfg)

    def forward(self, x, delta=None):
        return sum(self.forward_deferred(x, delta))

    def forward_deferred(self, x, delta=None):
        """(residual, mlp_out) with the block output = residual + mlp_out left unsummed, so the next
        LayerNorm adds it inside its kernel.  ``delta`` is the previous block's deferred mlp_out.
        (residual, LN(x)) come from one op: the residual-gradient add is fused into the LN backward."""
        if delta is None:
            x, h = T.layer_norm_residual(x, self.ln_1.weight, self.ln_1.bias, self.ln_1.eps)
        else:
            x, h = T.add_layer_norm_residual(x, delta, self.ln_1.weight, self.ln_1.bias, self.ln_1.eps)
        x, h = T.add_layer_norm_residual(x, self.attn(h), self.ln_2.weight, self.ln_2.bias, self.ln_2.eps)
        return x, self.mlp(h)


class _Transformer(tnn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.wte = tnn.Embedding(cfg.padded_vocab, cfg.n_embd)
        self.wpe = tnn.Embedding(cfg.block_size, cfg.n_embd)
        tnn.init.normal_(self.wte.weight, 0.0, 0.02)
        tnn.init.normal_(self.wpe.weight, 0.0, 0.01)
        self.h = tnn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = _LN(cfg.n_embd, cfg.ln_eps)


class GPT(tnn.Module):
    def __init__(self, cfg: GPTConfig = GPTConfig()):
        super().__init__()
        self.config = cfg
        self.transformer = _Transformer(cfg)

    def forward(self, idx, targets=None):
        t = self.transformer
        x = T.embedding(idx, t.wte.weight, t.wpe.weight)
        delta = None
        for blk in t.h:
            x, delta = blk.forward_deferred(x, delta)
        if delta is None:
            x = t.ln_f(x)
        else:   # last block's residual add fused into ln_f (the summed stream itself is not needed)
            x = T.add_layer_norm_residual(x, delta, t.ln_f.weight, t.ln_f.bias, t.ln_f.eps)[1]
        if targets is None:
            return T.lm_logits(x, t.wte.weight, self.config.vocab_size)
        return T.lm_head_loss(x, t.wte.weight, targets, self.config.vocab_size)

    def num_params(self, non_embedding: bool = False):
        n = sum(p.numel() for p in self.parameters())
        if non_embedding:
            n -= self.transformer.wpe.weight.numel()
        return n

    def decay_groups(self, weight_decay: float):
        """AdamW groups: matrices/embeddings decay, biases and LayerNorm parameters do not."""
        decay = [p for n, p in self.named_parameters() if p.dim() >= 2]
        nodecay = [p for n, p in self.named_parameters() if p.dim() < 2]
        return [{"params": decay, "weight_decay": weight_decay}, {"params": nodecay, "weight_decay": 0.0}]

    def flops_per_token(self) -> float:
        """Training FLOPs per token (6N for the matmul weights + causal attention, PaLM appendix B)."""
        c = self.config
        N = self.num_params() - self.transformer.wpe.weight.numel()
        return 6 * N + 6 * c.n_layer * c.n_embd * c.block_size  # causal: half of 12*L*C*T


def build_gpt2(cfg: GPTConfig = None, seed: int = 0, device=None, dtype=torch.bfloat16) -> GPT:
    torch.manual_seed(seed)
    m = GPT(cfg or GPTConfig())
    return m.to(device=device, dtype=dtype)
