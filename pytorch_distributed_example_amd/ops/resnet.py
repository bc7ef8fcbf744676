"""ResNet ops: training-mode BatchNorm fused with the residual add and ReLU (HIP kernels of
``csrc/kernels/resnet.hip``) over channels-last bf16 activations.

Forward:  y = relu(bn(x) + res)   -- 3 launches: partial stats, per-channel finalize (+ running-stat
          update), one streaming apply pass.
Backward: dy' = dy * (y > 0); dres = dy'; dx = BN backward of dy'  -- reduce, finalize (writes
          dgamma / dbeta), one streaming apply pass that also emits dres.
Convolutions with C_in, C_out multiples of 64 and kernels up to 3x3 (every ResNet-18 conv but the
3-channel stem) are implicit GEMMs on bf16 MFMA (``csrc/kernels/conv.hip``): fprop, phase-split
dgrad and split-K wgrad; the stem has its own MFMA kernels (``csrc/kernels/stem.hip``).  A GPU
convolution outside both raises (no silent MIOpen fallback); CPU tensors use the PyTorch reference
definitions.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._ext import kernels
from ..parallel.flat import flat_grad_slot


class BatchNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, run_mean, run_var, momentum, eps, relu, training, stats=None):
        K = kernels()
        C = x.shape[1]
        M = x.numel() // C
        dev = x.device
        y = torch.empty_like(x)
        mean = torch.empty(C, device=dev, dtype=torch.float32)
        rstd = torch.empty(C, device=dev, dtype=torch.float32)
        scale = torch.empty(C, device=dev, dtype=torch.float32)
        shift = torch.empty(C, device=dev, dtype=torch.float32)
        pre_nblk = 0
        if training and stats is not None:
            part, pre_nblk = stats                       # partial sums from the conv epilogue
        elif training:
            part = torch.empty(K.bn_blocks(M, C) * 2 * C, device=dev, dtype=torch.float32)
        else:
            part = torch.empty(0, device=dev, dtype=torch.float32)
            with torch.no_grad():                        # eval: fold running stats into scale / shift
                r = torch.rsqrt(run_var + eps)
                scale.copy_(gamma.float() * r)
                shift.copy_(beta.float() - run_mean * gamma.float() * r)
                mean.copy_(run_mean)
                rstd.copy_(r)
        K.bn_fwd(x, res, y, gamma, beta, eps, momentum, run_mean if training else None,
                 run_var if training else None, part, mean, rstd, scale, shift, relu, training, pre_nblk)
        ctx.save_for_backward(x, y, gamma, beta, mean, rstd)
        ctx.relu, ctx.has_res = relu, res is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, gamma, beta, mean, rstd = ctx.saved_tensors
        K = kernels()
        C = x.shape[1]
        M = x.numel() // C
        dev = x.device
        dy = dy.contiguous(memory_format=torch.channels_last) if dy.dim() == 4 else dy.contiguous()
        part = torch.empty(K.bn_blocks(M, C) * 2 * C, device=dev, dtype=torch.float32)
        coef = torch.empty(3 * C, device=dev, dtype=torch.float32)
        dgamma = flat_grad_slot(gamma)
        dgamma = torch.empty(C, device=dev, dtype=gamma.dtype) if dgamma is None else dgamma
        dbeta = flat_grad_slot(beta)
        dbeta = torch.empty(C, device=dev, dtype=gamma.dtype) if dbeta is None else dbeta
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if ctx.has_res else None
        K.bn_bwd(dy, y, x, gamma, mean, rstd, part, coef, dgamma, dbeta, dx, dres, ctx.relu)
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None, None


class Conv2dNHWCFn(torch.autograd.Function):
    """Bias-free conv2d over channels-last bf16 on the implicit-GEMM MFMA kernels."""

    @staticmethod
    def forward(ctx, x, w, stride, pad, with_stats=False):
        K = kernels()
        N, C, H, W = x.shape
        O, _, R, S = w.shape
        OH, OW = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
        y = torch.empty(N, O, OH, OW, device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
        stats = None
        if with_stats:
            nblk = K.conv_stats_blocks(N * OH * OW, O)
            stats = torch.empty(K.bn_part_rows(nblk) * 2 * O, device=x.device, dtype=torch.float32)
            ctx.nblk = nblk
            ctx.mark_non_differentiable(stats)
            ctx.set_materialize_grads(False)
        K.conv_fprop(x, w, y, stats, stride, pad)
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.pad = stride, pad
        return (y, stats) if with_stats else y

    @staticmethod
    def backward(ctx, dy, dstats=None):
        x, w = ctx.saved_tensors
        if dy is None:
            return None, None, None, None, None
        K = kernels()
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            wt = torch.empty(w.numel(), device=w.device, dtype=w.dtype)
            K.conv_dgrad(dy, w, wt, dx, ctx.stride, ctx.pad)
        if ctx.needs_input_grad[1]:
            splits = K.conv_wgrad_splits(x, w, ctx.stride, ctx.pad)
            part = torch.empty(splits * w.numel(), device=w.device, dtype=torch.float32)
            dw = flat_grad_slot(w)
            if dw is None or not dw.is_contiguous(memory_format=torch.channels_last):
                dw = torch.empty_like(w, memory_format=torch.channels_last)
            K.conv_wgrad(dy, x, w, part, splits, dw, ctx.stride, ctx.pad)
        return dx, dw, None, None, None


class StemConvFn(torch.autograd.Function):
    """ResNet stem conv (7x7 / s2 / p3, 3 -> 64) over channels-last bf16 on the stem MFMA kernel
    (csrc/kernels/stem.hip), optionally with the following BN's batch statistics."""

    @staticmethod
    def forward(ctx, x, w, with_stats=False):
        K = kernels()
        N, _, H, W = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty(N, 64, OH, OW, device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
        wp = torch.empty(64 * 224, device=x.device, dtype=x.dtype)
        stats = None
        if with_stats:
            nblk = K.stem_stats_blocks(N, OH)
            stats = torch.empty(K.bn_part_rows(nblk) * 2 * 64, device=x.device, dtype=torch.float32)
            ctx.nblk = nblk
            ctx.mark_non_differentiable(stats)
            ctx.set_materialize_grads(False)
        K.stem_fwd(x, w, wp, y, stats)
        ctx.save_for_backward(x, w)
        return (y, stats) if with_stats else y

    @staticmethod
    def backward(ctx, dy, dstats=None):
        x, w = ctx.saved_tensors
        if dy is None:
            return None, None, None
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:      # the network input never needs a gradient
            raise NotImplementedError("stem conv: no input-gradient kernel (the image input of ResNet-18 "
                                      "never requires grad)")
        if ctx.needs_input_grad[1]:
            K = kernels()
            part = torch.empty(K.stem_wgrad_blocks(x.shape[0], dy.shape[2]) * 64 * 147, device=x.device,
                               dtype=torch.float32)
            dw = flat_grad_slot(w)
            if dw is None or not dw.is_contiguous(memory_format=torch.channels_last):
                dw = torch.empty_like(w, memory_format=torch.channels_last)
            K.stem_wgrad(x, dy, part, dw)
        return dx, dw, None


def stem_eligible(x, w, stride: int, pad: int) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and x.shape[1] == 3 and tuple(w.shape) == (64, 3, 7, 7) and stride == 2 and pad == 3
            and (x.shape[3] - 1) // 2 + 1 <= 112)


def igemm_eligible(x, w, stride: int, pad: int) -> bool:
    """True when the MFMA implicit-GEMM kernels cover this convolution."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0 and w.shape[2] * w.shape[3] <= 9
            and stride in (1, 2) and 0 <= pad < w.shape[2])


def conv2d_nhwc(x, w, stride: int = 1, pad: int = 0, with_stats: bool = False):
    """conv2d (no bias) for channels-last bf16 activations: MFMA implicit GEMM where eligible.
    ``with_stats``: return ``(y, stats)`` where ``stats`` is ``(partials, nblk)`` -- per-channel
    (sum, sum of squares) partials of y for a following training-mode BatchNorm -- or None when
    the library path ran."""
    if stem_eligible(x, w, stride, pad):
        out = StemConvFn.apply(x.contiguous(memory_format=torch.channels_last),
                               w.contiguous(memory_format=torch.channels_last), with_stats)
        if with_stats:
            y, part = out
            return y, (part, kernels().stem_stats_blocks(y.shape[0], y.shape[2]))
        return out
    if igemm_eligible(x, w, stride, pad):
        out = Conv2dNHWCFn.apply(x.contiguous(memory_format=torch.channels_last),
                                 w.contiguous(memory_format=torch.channels_last), stride, pad, with_stats)
        if with_stats:
            y, part = out
            return y, (part, kernels().conv_stats_blocks(y.shape[0] * y.shape[2] * y.shape[3], w.shape[0]))
        return out
    if x.is_cuda:
        # no silent library fallback on the GPU: every ResNet-18 convolution is covered above
        raise NotImplementedError(
            f"conv2d_nhwc: no MFMA kernel for x {tuple(x.shape)} {x.dtype}, w {tuple(w.shape)}, stride {stride}, "
            f"pad {pad} (implicit GEMM needs C_in, C_out multiples of 64, <= 3x3 taps, stride 1/2; the stem "
            f"kernel covers 3->64 7x7/s2/p3)")
    y = F.conv2d(x, w, None, stride, pad)
    return (y, None) if with_stats else y


def batch_norm_act(x, gamma, beta, running_mean, running_var, training: bool, momentum: float = 0.1,
                   eps: float = 1e-5, residual=None, relu: bool = True, stats=None):
    """``stats``: optional ``(partials, nblk)`` from ``conv2d_nhwc(..., with_stats=True)`` (the batch
    statistics of ``x`` were summed by the convolution that produced it)."""
    if x.is_cuda:
        if x.dim() == 4 and not x.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        if residual is not None and residual.dim() == 4:
            residual = residual.contiguous(memory_format=torch.channels_last)
        return BatchNormActFn.apply(x, gamma, beta, residual, running_mean, running_var, momentum, eps, relu,
                                    training, stats if training else None)
    y = F.batch_norm(x, running_mean, running_var, gamma, beta, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class MaxPool3s2Fn(torch.autograd.Function):
    """3x3 / stride 2 / pad 1 max-pool over channels-last bf16 (ResNet stem)."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty(N, C, OH, OW, device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
        arg = torch.empty(y.numel(), device=x.device, dtype=torch.uint8)
        kernels().maxpool3s2_fwd(x, y, arg)
        ctx.save_for_backward(arg)
        ctx.xshape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        N, C, H, W = ctx.xshape
        dx = torch.empty(N, C, H, W, device=dy.device, dtype=dy.dtype, memory_format=torch.channels_last)
        kernels().maxpool3s2_bwd(dy.contiguous(memory_format=torch.channels_last), arg, dx)
        return dx


def max_pool3s2(x):
    if x.is_cuda and x.dim() == 4 and x.shape[1] % 8 == 0:
        return MaxPool3s2Fn.apply(x.contiguous(memory_format=torch.channels_last))
    return F.max_pool2d(x, 3, 2, 1)
