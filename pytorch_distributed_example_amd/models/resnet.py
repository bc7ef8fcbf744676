"""ResNet-18 (bf16, channels-last) -- driver-added config of BASELINE.json ("ResNet-18 bf16 on
synthetic 3x224x224, DDP 8xMI355X").  Same architecture / parameter names as torchvision's
``resnet18`` (conv1/bn1, layer1..layer4 of BasicBlocks with downsample, fc), so state_dicts
interchange; BatchNorm+residual+ReLU run as fused HIP kernels (``ops.resnet``); every convolution except the 3-channel
stem is an implicit GEMM on bf16 MFMA (``csrc/kernels/conv.hip``), the stem has its own MFMA kernels
(``csrc/kernels/stem.hip``); a training BasicBlock is one autograd node (``ops.resnet.BasicBlockFn``:
residual-gradient add inside conv1's dgrad epilogue); the head is an own pool kernel + the own GEMM.
"""
from __future__ import annotations

import math

import torch
import torch.nn as tnn

from ..ops.resnet import (DgradWeights, basic_block_eligible, basic_block_train, batch_norm_act, bn_relu_maxpool,
                          conv2d_nhwc, max_pool3s2, resnet_head)


class BN(tnn.Module):
    """BatchNorm2d with torchvision's parameter / buffer names; running stats stay fp32."""

    def __init__(self, C, momentum=0.1, eps=1e-5, zero_init=False):
        super().__init__()
        self.weight = tnn.Parameter(torch.zeros(C) if zero_init else torch.ones(C))
        self.bias = tnn.Parameter(torch.zeros(C))
        self.register_buffer("running_mean", torch.zeros(C))
        self.register_buffer("running_var", torch.ones(C))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        self.momentum, self.eps = momentum, eps

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        # keep running statistics fp32 when the module is cast to bf16
        self.running_mean.data = self.running_mean.data.float()
        self.running_var.data = self.running_var.data.float()
        return self

    def forward(self, x, residual=None, relu=True, stats=None):
        if isinstance(x, tuple):                 # (conv output, its fused BN partial sums)
            x, stats = x
        if self.training and not getattr(self, "_counted_by_model", False):
            self.num_batches_tracked.add_(1)
        return batch_norm_act(x, self.weight, self.bias, self.running_mean, self.running_var, self.training,
                              self.momentum, self.eps, residual, relu, stats)


class Conv2d(tnn.Conv2d):
    """torch Conv2d (same parameter name / layout / init) whose forward runs the MFMA implicit GEMM."""

    def forward(self, x, with_stats: bool = False):
        """``with_stats`` (the conv feeds a training-mode BN): returns ``(y, stats)``."""
        return conv2d_nhwc(x, self.weight, self.stride[0], self.padding[0], with_stats)


def _conv(cin, cout, k, stride=1, pad=0):
    c = Conv2d(cin, cout, k, stride, pad, bias=False)
    tnn.init.kaiming_normal_(c.weight, mode="fan_out", nonlinearity="relu")
    return c


class BasicBlock(tnn.Module):
    expansion = 1

    def __init__(self, cin, cout, stride=1, zero_init_residual=False):
        super().__init__()
        self.conv1 = _conv(cin, cout, 3, stride, 1)
        self.bn1 = BN(cout)
        self.conv2 = _conv(cout, cout, 3, 1, 1)
        self.bn2 = BN(cout, zero_init=zero_init_residual)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = tnn.Sequential(_conv(cin, cout, 1, stride), BN(cout))

    def forward(self, x):
        st = self.training and x.is_cuda
        if st and basic_block_eligible(x, self.conv1.weight, self.conv2.weight, None):
            # one autograd node: residual-gradient add fused into conv1's dgrad epilogue
            ds = self.downsample
            return basic_block_train(x, self.conv1, self.bn1, self.conv2, self.bn2,
                                     ds[0] if ds is not None else None, ds[1] if ds is not None else None)
        if self.downsample is not None:
            idt = self.downsample[1](self.downsample[0](x, st), relu=False)
        else:
            idt = x
        out = self.bn1(self.conv1(x, st))
        return self.bn2(self.conv2(out, st), residual=idt, relu=True)


class ResNet(tnn.Module):
    def __init__(self, layers=(2, 2, 2, 2), num_classes=1000, zero_init_residual=False):
        super().__init__()
        self.conv1 = _conv(3, 64, 7, 2, 3)
        self.bn1 = BN(64)
        widths = (64, 128, 256, 512)
        cin = 64
        for i, (w, n) in enumerate(zip(widths, layers)):
            blocks = []
            for j in range(n):
                blocks.append(BasicBlock(cin, w, 2 if (j == 0 and i > 0) else 1, zero_init_residual))
                cin = w
            setattr(self, f"layer{i + 1}", tnn.Sequential(*blocks))
        self.fc = tnn.Linear(512, num_classes)
        bound = 1 / math.sqrt(512)
        tnn.init.uniform_(self.fc.weight, -bound, bound)
        tnn.init.uniform_(self.fc.bias, -bound, bound)

    def _bn_counters(self):
        """All BN ``num_batches_tracked`` buffers as views of one int64 tensor, so a training forward
        bumps them with one launch instead of 20 (re-linked after ``.to()`` / buffer replacement)."""
        bns = [m for m in self.modules() if isinstance(m, BN)]
        sh = self.__dict__.get("_nbt_shared")
        ok = sh is not None and sh.device == bns[0].num_batches_tracked.device and all(
            b.num_batches_tracked.data_ptr() == sh.data_ptr() + i * sh.element_size() for i, b in enumerate(bns))
        if not ok:
            sh = torch.stack([b.num_batches_tracked.detach() for b in bns])
            for i, b in enumerate(bns):
                b._buffers["num_batches_tracked"] = sh[i]
                b._counted_by_model = True
            self.__dict__["_nbt_shared"] = sh
        return sh

    def _dgrad_weights(self):
        """Every block convolution weight whose input gradient the backward computes (all but the stem),
        in a fixed order, for the one batched transpose launch per training forward."""
        ws = []
        for i in range(1, 5):
            for blk in getattr(self, f"layer{i}"):
                ws += [blk.conv1.weight, blk.conv2.weight]
                if blk.downsample is not None:
                    ws.append(blk.downsample[0].weight)
        return ws

    def forward(self, x):
        counted = False
        if self.training and x.is_cuda:
            ws = self._dgrad_weights()
            if all(w.is_contiguous(memory_format=torch.channels_last) and w.shape[0] % 64 == 0
                   and w.shape[1] % 64 == 0 for w in ws):
                # the batched dgrad-weight transpose launch also bumps the BN counters
                self.__dict__.setdefault("_wt_cache", DgradWeights()).refresh(ws, self._bn_counters())
                counted = True
        if self.training and not counted:
            self._bn_counters().add_(1)
        if self.training and x.is_cuda:
            # stem BN + ReLU + max-pool as one fused node: the 64x112x112 post-BN map is never stored
            y, stats = self.conv1(x, True)
            x = bn_relu_maxpool(y, stats, self.bn1)
        else:
            x = max_pool3s2(self.bn1(self.conv1(x, False)))
        for i in range(1, 5):
            x = getattr(self, f"layer{i}")(x)
        return resnet_head(x, self.fc.weight, self.fc.bias)

    def decay_groups(self, weight_decay: float):
        """SGD groups: conv / fc weights decay; BN parameters and biases do not."""
        decay = [p for n, p in self.named_parameters() if p.dim() > 1]
        nodecay = [p for n, p in self.named_parameters() if p.dim() <= 1]
        return [{"params": decay, "weight_decay": weight_decay}, {"params": nodecay, "weight_decay": 0.0}]


def build_resnet18(num_classes=1000, seed=0, device=None, dtype=torch.bfloat16) -> ResNet:
    torch.manual_seed(seed)
    m = ResNet((2, 2, 2, 2), num_classes)
    m = m.to(device=device, dtype=dtype)
    if device is not None and torch.device(device).type == "cuda":
        m = m.to(memory_format=torch.channels_last)
    return m
