"""Fused forward/backward of the reference toy CNN as one autograd Function (HIP kernels).

``Net.forward`` (/root/reference/mnist/main.py:139-147) is
  relu(conv1) -> maxpool2 -> relu(conv2) -> maxpool2 -> view(-1, 800) -> relu(fc1) -> fc2 -> log_softmax
and is executed here by the fused kernels of ``csrc/kernels/lenet_v2.hip`` / ``lenet.hip``: the v2
conv forward (LDS-DMA weight staging, 8-wave MFMA conv1 + conv2) for every batch size, fc1, the
one-row-per-block head, and in backward the fc backward plus the v2 conv backward with the "ext"
reduction (slabs and per-image conv1 partials, folded in fixed order by k_conv_grad_fold) for
B <= 128; only batches above 128 take lenet.hip's first-generation conv backward.  The function
returns log-probabilities exactly like the reference model, so any loss can follow it; the training
engine (``engine/lenet.py``) additionally fuses the loss and runs the whole step without autograd.
"""
from __future__ import annotations

import torch

from .._ext import kernels


class LeNetWorkspace:
    """Per-(device, batch) activation buffers kept between forward and backward."""

    def __init__(self, B: int, device):
        f32 = dict(device=device, dtype=torch.float32)
        self.B = B
        self.P1 = torch.empty(B * 2880, **f32)
        self.A1 = torch.empty(B * 2880, device=device, dtype=torch.uint8)
        self.P2 = torch.empty(B * 800, **f32)
        self.A2 = torch.empty(B * 800, device=device, dtype=torch.uint8)
        self.H1 = torch.empty(B * 500, **f32)
        self.dZ1 = torch.empty(B * 500, **f32)
        self.dZ2 = torch.empty(B * 10, **f32)
        self.dP2m = torch.empty(B * 800, **f32)
        self.rows = torch.arange(B, device=device, dtype=torch.int32)
        self.Wp = torch.zeros(2 * 72 * 256, **f32)       # v2 conv2 weight image (padding stays zero)


def _bwd2_scratch(ws: "LeNetWorkspace"):
    """Reduction scratch of the v2 conv backward ("ext" mode): 16 conv2 slabs, per-image conv1
    partials, and the fold-mode buffers the kernel signature carries (unused here).  Owned by the
    forward's workspace (``ctx.ws``), like ``Wp``: two backwards in flight at once (two models,
    side streams, graph capture on different streams) never share a slab."""
    sc = getattr(ws, "bwd2_scratch", None)
    if sc is None:
        f32 = dict(device=ws.P1.device, dtype=torch.float32)
        sc = {"slab": torch.zeros(16 * 25088, **f32), "c1img": torch.zeros(ws.B * 520, **f32),
              "c1rep": torch.zeros(16 * 576, device=ws.P1.device, dtype=torch.int64),
              "c1part": torch.zeros(16 * 576, **f32), "tick": torch.zeros(32, device=ws.P1.device, dtype=torch.int32)}
        ws.bwd2_scratch = sc
    return sc


def pack_conv2_weight(w2: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """[50,20,5,5] -> [500 (k'=(kh*5+kw)*20+ci)][64 (co, zero padded)] layout of the conv2 kernel."""
    if out is None:
        out = torch.empty(500 * 64, device=w2.device, dtype=torch.float32)
    kernels().lenet_pack_w2(w2.detach().contiguous(), out)
    return out


class LeNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1c, b1c, w2c, b2c, w1f, b1f, w2f, b2f):
        K = kernels()
        B = x.shape[0]
        dev = x.device
        ws = LeNetWorkspace(B, dev)
        xf = x.detach().reshape(B, 784).contiguous()
        if xf.dtype != torch.float32:
            raise TypeError("LeNet fused path is fp32 (the reference model's dtype)")
        K.lenet_pack_w2_v2(w2c.detach().contiguous(), ws.Wp)
        K.lenet_conv_fwd2(xf, B, w1c.detach().contiguous(), b1c.detach().contiguous(), ws.Wp,
                          b2c.detach().contiguous(), ws.P1, ws.A1, ws.P2, ws.A2)
        K.lenet_fc1_fwd(ws.P2, B, w1f.detach().contiguous(), b1f.detach().contiguous(), ws.H1, None)
        logp = torch.empty(B, 10, device=dev, dtype=torch.float32)
        dummy = torch.zeros(B, device=dev, dtype=torch.long)
        K.lenet_head(ws.H1, B, w2f.detach().contiguous(), b2f.detach().contiguous(), dummy, 1.0 / B, logp,
                     None, None, None, None, None, None)
        ctx.ws = ws
        ctx.save_for_backward(xf, w2c, w1f, w2f, logp)
        ctx.x_needs_grad = x.requires_grad
        return logp

    @staticmethod
    def backward(ctx, g_logp):
        if ctx.x_needs_grad:
            raise NotImplementedError("fused LeNet backward does not produce d(input) (conv1 dgrad)")
        K = kernels()
        xf, w2c, w1f, w2f, logp = ctx.saved_tensors
        ws = ctx.ws
        B = ws.B
        dev = xf.device
        K.lenet_head_bwd(ws.H1, B, w2f.detach().contiguous(), logp, g_logp.contiguous().float(), ws.dZ2, ws.dZ1)
        grads = torch.zeros(431080, device=dev, dtype=torch.float32)
        o = 0
        views = []
        for n, shp in ((500, (20, 1, 5, 5)), (20, (20,)), (25000, (50, 20, 5, 5)), (50, (50,)), (400000, (500, 800)),
                       (500, (500,)), (5000, (10, 500)), (10, (10,))):
            views.append(grads[o:o + n].view(shp))
            o += n
        gw1c, gb1c, gw2c, gb2c, gw1f, gb1f, gw2f, gb2f = views
        K.lenet_fc_bwd(ws.P2, ws.H1, ws.dZ1, ws.dZ2, w1f.detach().contiguous(), B, ws.dP2m, gw1f, gb1f, gw2f, gb2f,
                       None, None, None, None)
        if B <= 128:
            sc = _bwd2_scratch(ws)
            c1w, c1b, c2w, c2b = 0, 500, 520, 25520           # flat offsets of the views above
            K.lenet_conv_bwd2(xf, ws.P1, ws.A1, ws.dP2m, ws.A2, w2c.detach().contiguous(), B, sc["slab"], sc["c1rep"],
                              sc["c1part"], sc["tick"], grads, c1w, c1b, c2w, c2b, defer=2, c1img=sc["c1img"])
            K.lenet_conv_grad_fold(sc["slab"], sc["c1img"], B, grads, c1w, c1b, c2w, c2b)
        else:
            K.lenet_conv_bwd(xf, ws.rows, ws.P1, ws.A1, ws.dP2m, ws.A2, w2c.detach().contiguous(), B, gw1c, gb1c,
                             gw2c, gb2c)
        return None, gw1c, gb1c, gw2c, gb2c, gw1f, gb1f, gw2f, gb2f


def lenet_forward(x, net):
    return LeNetFunction.apply(x, net.conv1.weight, net.conv1.bias, net.conv2.weight, net.conv2.bias,
                               net.fc1.weight, net.fc1.bias, net.fc2.weight, net.fc2.bias)
