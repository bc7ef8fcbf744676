"""Generic GPU ops (autograd Functions) over the HIP kernels of ``csrc/kernels/generic.hip``.

Every forward and backward of Linear / Conv2d / ReLU / 2x2 MaxPool / log_softmax / cross_entropy
runs a framework kernel (fp32 MFMA GEMM with fused bias/ReLU epilogues, im2col/col2im, row-wise
softmax kernels).  Output allocation uses torch's caching allocator; no ATen compute kernels are
used for these ops (the only exception is the final 1/B scaling of a mean loss scalar).
"""
from __future__ import annotations

import torch

from .._ext import kernels


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def _gemm(A, B, C, M, N, K, lda, ldb, ldc, transA=False, transB=False, bias=None, bias_mode=0, relu=False,
          beta=0.0, batch=1, sA=0, sB=0, sC=0, atomic=False):
    kernels().gemm(A, B, C, bias, M, N, K, lda, ldb, ldc, transA, transB, sA, sB, sC, batch, 1.0, beta, bias_mode,
                   relu, atomic)


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        shp = x.shape
        x2 = _c(x.reshape(-1, shp[-1]))
        B, IN = x2.shape
        OUT = w.shape[0]
        wc = _c(w)
        y = torch.empty(B, OUT, device=x.device, dtype=torch.float32)
        _gemm(x2, wc, y, B, OUT, IN, IN, IN, OUT, transB=True, bias=b.detach() if b is not None else None,
              bias_mode=1 if b is not None else 0)
        ctx.save_for_backward(x2, wc)
        ctx.has_bias = b is not None
        ctx.shp = shp
        return y.reshape(*shp[:-1], OUT)

    @staticmethod
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        B, IN = x2.shape
        OUT = w.shape[0]
        g = _c(gy.reshape(-1, OUT).float())
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(B, IN, device=g.device, dtype=torch.float32)
            _gemm(g, w, dx, B, IN, OUT, OUT, IN, IN)
            dx = dx.reshape(ctx.shp)
        if ctx.needs_input_grad[1]:
            dw = torch.empty(OUT, IN, device=g.device, dtype=torch.float32)
            _gemm(g, x2, dw, OUT, IN, B, OUT, IN, IN, transA=True)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = torch.empty(OUT, device=g.device, dtype=torch.float32)
            kernels().colsum(g, B, OUT, db)
        return dx, dw, db


class ReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        xc = _c(x)
        y = torch.empty_like(xc)
        kernels().relu_fwd(xc, y)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        dx = torch.empty_like(y)
        kernels().relu_bwd(y, _c(g), dx)
        return dx


class LogSoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        xc = _c(x)
        out = torch.empty_like(xc)
        kernels().log_softmax_fwd(xc, out)
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, g):
        (out,) = ctx.saved_tensors
        dx = torch.empty_like(out)
        kernels().log_softmax_bwd(out, _c(g), dx)
        return dx


class CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, reduction):
        xc = _c(x)
        B, C = xc.shape
        yc = _c(y.to(torch.int64))
        rl = torch.empty(B, device=x.device, dtype=torch.float32)
        lse = torch.empty(B, device=x.device, dtype=torch.float32)
        kernels().xent_fwd(xc, yc, rl, lse)
        ctx.save_for_backward(xc, yc, lse)
        ctx.reduction = reduction
        if reduction == "none":
            return rl
        tot = torch.empty(1, device=x.device, dtype=torch.float32)
        kernels().sum_f32(rl, tot, 1.0 / B if reduction == "mean" else 1.0)   # the mean's divide folded in
        return tot.reshape(())

    @staticmethod
    def backward(ctx, g):
        xc, yc, lse = ctx.saved_tensors
        B = xc.shape[0]
        dx = torch.empty_like(xc)
        per_row = ctx.reduction == "none"
        mul = 1.0 / B if ctx.reduction == "mean" else 1.0
        gs = g.reshape(-1)
        if gs.dtype != torch.float32:
            gs = gs.float()
        kernels().xent_bwd(xc, yc, lse, _c(gs), per_row, mul, dx)
        return dx, None, None


class MaxPool2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        xc = _c(x)
        N, C, H, W = xc.shape
        y = torch.empty(N, C, H // 2, W // 2, device=x.device, dtype=torch.float32)
        code = torch.empty(N, C, H // 2, W // 2, device=x.device, dtype=torch.uint8)
        kernels().pool2_fwd(xc, N * C, H, W, y, code)
        ctx.save_for_backward(code)
        ctx.shp = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, g):
        (code,) = ctx.saved_tensors
        N, C, H, W = ctx.shp
        dx = torch.empty(N, C, H, W, device=g.device, dtype=torch.float32)
        kernels().pool2_bwd(_c(g), code, N * C, H, W, dx)
        return dx


class Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad):
        xc = _c(x)
        N, C, H, W = xc.shape
        O, _, KH, KW = w.shape
        OH = (H + 2 * pad - KH) // stride + 1
        OW = (W + 2 * pad - KW) // stride + 1
        R, P = C * KH * KW, OH * OW
        col = torch.empty(N, R, P, device=x.device, dtype=torch.float32)
        K = kernels()
        K.im2col(xc, N, C, H, W, KH, KW, stride, pad, OH, OW, col)
        y = torch.empty(N, O, OH, OW, device=x.device, dtype=torch.float32)
        wm = _c(w.reshape(O, R))
        _gemm(wm, col, y, O, P, R, R, P, P, bias=b.detach() if b is not None else None,
              bias_mode=2 if b is not None else 0, batch=N, sA=0, sB=R * P, sC=O * P)
        ctx.save_for_backward(col, wm)
        ctx.meta = (N, C, H, W, O, KH, KW, OH, OW, stride, pad, b is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        col, wm = ctx.saved_tensors
        N, C, H, W, O, KH, KW, OH, OW, stride, pad, has_b = ctx.meta
        R, P = C * KH * KW, OH * OW
        g = _c(gy.float())
        K = kernels()
        dx = dw = db = None
        if ctx.needs_input_grad[1]:
            dw = torch.zeros(O, R, device=g.device, dtype=torch.float32)
            _gemm(g, col, dw, O, R, P, P, P, R, transB=True, batch=N, sA=O * P, sB=R * P, sC=0, atomic=True)
            dw = dw.reshape(O, C, KH, KW)
        if ctx.needs_input_grad[0]:
            dcol = torch.empty(N, R, P, device=g.device, dtype=torch.float32)
            _gemm(wm, g, dcol, R, P, O, R, P, P, transA=True, batch=N, sA=0, sB=O * P, sC=R * P)
            dx = torch.empty(N, C, H, W, device=g.device, dtype=torch.float32)
            K.col2im(dcol, N, C, H, W, KH, KW, stride, pad, OH, OW, dx)
        if has_b and ctx.needs_input_grad[2]:
            db = torch.empty(O, device=g.device, dtype=torch.float32)
            K.bias_grad_nchw(g, N, O, P, db)
        return dx, dw, db, None, None


def _f32(t, name):
    if t.dtype != torch.float32:
        raise TypeError(f"GPU op {name}: fp32 kernels only (got {t.dtype})")


def linear(x, weight, bias=None):
    _f32(x, "linear")
    return LinearFn.apply(x, weight, bias)


def relu(x):
    _f32(x, "relu")
    return ReluFn.apply(x)


def conv2d(x, weight, bias=None, stride=1, padding=0):
    _f32(x, "conv2d")
    s = stride if isinstance(stride, int) else stride[0]
    p = padding if isinstance(padding, int) else padding[0]
    return Conv2dFn.apply(x, weight, bias, s, p)


def max_pool2d(x, kernel_size=2, stride=2):
    ks = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
    st = stride if isinstance(stride, int) else (stride[0] if stride else ks)
    if ks != 2 or st != 2 or x.dim() != 4 or x.shape[-1] % 2 or x.shape[-2] % 2:
        raise NotImplementedError("GPU max_pool2d kernel: 2x2, stride 2, even H/W")
    return MaxPool2Fn.apply(x)


def log_softmax(x, dim=1):
    if x.dim() != 2 or dim not in (1, -1):
        raise NotImplementedError("GPU log_softmax kernel: 2-D input, dim=1")
    return LogSoftmaxFn.apply(x)


def cross_entropy(logits, target, reduction="mean"):
    if logits.dim() != 2:
        raise NotImplementedError("GPU cross_entropy kernel: [B, C] logits")
    if logits.dtype not in (torch.float32, torch.bfloat16):
        logits = logits.float()
    return CrossEntropyFn.apply(logits, target, reduction)          # bf16 logits read as they are
