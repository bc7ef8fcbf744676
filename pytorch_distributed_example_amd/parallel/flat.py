"""Flat parameter / gradient storage laid out in communication-bucket order.

All parameters of a module are re-homed into ONE contiguous fp32 buffer (``p.data`` becomes a view),
and all gradients into a second one (``p.grad`` is a view).  Buckets are contiguous ranges of
both buffers, so a bucket all-reduce is a single collective on a zero-copy view, and the fused
optimizer updates every parameter in one launch.  Each tensor starts on a 64-element (256 B)
boundary, so vectorised kernels and RCCL see aligned buffers.  A 4-D parameter that is
channels-last when bound keeps that layout: its slot stores [N][H][W][C] and every view of it
(parameter, gradient, optimizer state) carries channels-last strides, so NHWC kernels read the
weights in place and write weight gradients straight into the flat gradient buffer.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import torch

ALIGN = 64


@dataclass
class Slot:
    name: str
    offset: int
    numel: int
    shape: Tuple[int, ...]
    channels_last: bool = False


class FlatLayout:
    """``extra_shapes`` are non-parameter gradient slots (e.g. atomic-contention replicas) that take
    part in the buckets (and therefore in the all-reduce) but are never bound to a parameter."""

    def __init__(self, named_shapes: Sequence[Tuple[str, Tuple[int, ...]]], buckets: Sequence[Sequence[str]],
                 align: int = ALIGN, extra_shapes: Dict[str, Tuple[int, ...]] | None = None):
        shapes = dict(named_shapes)
        self.param_names = list(shapes)
        shapes.update(extra_shapes or {})
        seen = [n for b in buckets for n in b]
        if sorted(seen) != sorted(shapes):
            raise ValueError("buckets must partition the parameter set exactly")
        self.slots: Dict[str, Slot] = {}
        self.bucket_ranges: List[Tuple[int, int]] = []
        self.bucket_names: List[List[str]] = [list(b) for b in buckets]
        off = 0
        for b in buckets:
            start = off
            for n in b:
                shp = tuple(shapes[n])
                numel = 1
                for d in shp:
                    numel *= d
                self.slots[n] = Slot(n, off, numel, shp)
                off += (numel + align - 1) // align * align
            self.bucket_ranges.append((start, off))
        self.total = off

    @classmethod
    def for_module(cls, module: torch.nn.Module, buckets=None, bucket_cap_bytes: int | None = None):
        named = [(n, tuple(p.shape)) for n, p in module.named_parameters() if p.requires_grad]
        if buckets is None:
            buckets = reverse_order_buckets(named, bucket_cap_bytes or (25 << 20))
        return cls(named, buckets)

    def bind(self, module, device=None, dtype=torch.float32):
        """Move parameters (a module or a {name: param} dict) into flat storage; returns
        (flat_params, flat_grads).  Each parameter is tagged ``p._pde_flat = (layout, flat_params,
        flat_grads, name)`` so DDP and the fused optimizers can share one buffer."""
        params = dict(module.named_parameters()) if isinstance(module, torch.nn.Module) else dict(module)
        dev = device or next(iter(params.values())).device
        flat_p = torch.zeros(self.total, device=dev, dtype=dtype)
        flat_g = torch.zeros(self.total, device=dev, dtype=dtype)
        for n, s in self.slots.items():
            if n not in self.param_names:
                continue
            p = params[n]
            s.channels_last = (p.dim() == 4 and not p.is_contiguous()
                               and p.is_contiguous(memory_format=torch.channels_last))
            v = self.view(flat_p, n)
            v.copy_(p.detach())
            p.data = v
            gv = self.view(flat_g, n)
            if p.grad is not None:          # binding after a backward (lazy optimizer init): keep the grad
                gv.copy_(p.grad.detach())
            p.grad = gv
            p._pde_flat = (self, flat_p, flat_g, n)
        return flat_p, flat_g

    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        s = self.slots[name]
        v = flat[s.offset: s.offset + s.numel]
        if s.channels_last:
            n, c, h, w = s.shape
            return v.view(n, h, w, c).permute(0, 3, 1, 2)
        return v.view(s.shape)

    def bucket_view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        a, b = self.bucket_ranges[i]
        return flat[a:b]


def reverse_order_buckets(named_shapes, cap_bytes: int, elem_bytes: int = 4):
    """DDP-style buckets: parameters in REVERSE registration order (gradients become ready roughly
    in that order during backward), greedily packed up to ``cap_bytes`` per bucket."""
    buckets, cur, cur_bytes = [], [], 0
    for n, shp in reversed(list(named_shapes)):
        numel = 1
        for d in shp:
            numel *= d
        nb = numel * elem_bytes
        if cur and cur_bytes + nb > cap_bytes:
            buckets.append(cur)
            cur, cur_bytes = [], 0
        cur.append(n)
        cur_bytes += nb
    if cur:
        buckets.append(cur)
    return buckets


def flat_grad_slot(p: torch.Tensor):
    """Where an op should write ``p``'s gradient: a fresh view of ``p``'s flat gradient slot (same
    shape and strides as ``p``) when ``p`` is flat-bound and has no gradient yet, else None.  The op
    overwrites the whole view and returns it; autograd then adopts it as ``p.grad`` without a copy
    (``AccumulateGrad`` steals a layout-matching gradient), so DDP buckets and the fused optimizers
    see it in place."""
    tag = getattr(p, "_pde_flat", None)
    if tag is None or p.grad is not None:
        return None
    layout, _, fg, name = tag
    return layout.view(fg, name)


def shared_flat(params):
    """If every parameter in ``params`` is bound to the same flat buffer (and it covers exactly
    them), return (layout, flat_params, flat_grads); else None."""
    tags = [getattr(p, "_pde_flat", None) for p in params]
    if not tags or any(t is None for t in tags):
        return None
    layout, fp, fg = tags[0][0], tags[0][1], tags[0][2]
    if any(t[0] is not layout for t in tags):
        return None
    if sorted(t[3] for t in tags) != sorted(layout.param_names):
        return None
    for p, t in zip(params, tags):
        s = layout.slots[t[3]]
        if p.data_ptr() != fp[s.offset:].data_ptr():
            return None
    return layout, fp, fg
