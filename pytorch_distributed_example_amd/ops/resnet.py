"""ResNet ops: training-mode BatchNorm fused with the residual add and ReLU (HIP kernels of
``csrc/kernels/resnet.hip``) over channels-last bf16 activations.

Forward:  y = relu(bn(x) + res)   -- 3 launches: partial stats, per-channel finalize (+ running-stat
          update), one streaming apply pass.
Backward: dy' = dy * (y > 0); dres = dy'; dx = BN backward of dy'  -- reduce, finalize (writes
          dgamma / dbeta), one streaming apply pass that also emits dres.
The convolutions themselves are library convolutions (MIOpen through ``torch.nn.functional.conv2d``
on channels-last bf16 tensors); CPU tensors use the PyTorch reference definition.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._ext import kernels


class BatchNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, run_mean, run_var, momentum, eps, relu, training):
        K = kernels()
        C = x.shape[1]
        M = x.numel() // C
        dev = x.device
        y = torch.empty_like(x)
        mean = torch.empty(C, device=dev, dtype=torch.float32)
        rstd = torch.empty(C, device=dev, dtype=torch.float32)
        scale = torch.empty(C, device=dev, dtype=torch.float32)
        shift = torch.empty(C, device=dev, dtype=torch.float32)
        if training:
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
                 run_var if training else None, part, mean, rstd, scale, shift, relu, training)
        ctx.save_for_backward(x, y, gamma, mean, rstd)
        ctx.relu, ctx.has_res = relu, res is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, gamma, mean, rstd = ctx.saved_tensors
        K = kernels()
        C = x.shape[1]
        M = x.numel() // C
        dev = x.device
        dy = dy.contiguous(memory_format=torch.channels_last) if dy.dim() == 4 else dy.contiguous()
        part = torch.empty(K.bn_blocks(M, C) * 2 * C, device=dev, dtype=torch.float32)
        coef = torch.empty(3 * C, device=dev, dtype=torch.float32)
        dgamma = torch.empty(C, device=dev, dtype=gamma.dtype)
        dbeta = torch.empty(C, device=dev, dtype=gamma.dtype)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if ctx.has_res else None
        K.bn_bwd(dy, y, x, gamma, mean, rstd, part, coef, dgamma, dbeta, dx, dres, ctx.relu)
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None


def batch_norm_act(x, gamma, beta, running_mean, running_var, training: bool, momentum: float = 0.1,
                   eps: float = 1e-5, residual=None, relu: bool = True):
    if x.is_cuda:
        if x.dim() == 4 and not x.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        if residual is not None and residual.dim() == 4:
            residual = residual.contiguous(memory_format=torch.channels_last)
        return BatchNormActFn.apply(x, gamma, beta, residual, running_mean, running_var, momentum, eps, relu,
                                    training)
    y = F.batch_norm(x, running_mean, running_var, gamma, beta, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y
