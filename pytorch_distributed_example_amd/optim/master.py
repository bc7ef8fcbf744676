"""Optimizers for bf16 models with fp32 master weights: one fused HIP launch per step.

The model's parameters are bf16 (what the GEMMs / convolutions and the gradient all-reduce move);
these optimizers own fp32 master copies and their moment buffers as flat buffers aligned with the
parameters' flat layout (shared with DDP's buckets when the model is wrapped first), so an update is
one streaming pass with no host synchronisation:

* ``AdamWMaster``: g = grad * grad_scale * min(1, max_norm / ||grad||) (global-norm clipping computed
  on device), decoupled weight decay, torch.optim.AdamW math; writes p32 and bf16(p32).  With
  ``capturable=True`` the step count lives on the device, so the whole step can be a hipGraph.
* ``SGDMaster``:   torch.optim.SGD math (momentum, coupled weight decay, optional nesterov).

Per-group weight decay is a per-64-element flag table (every parameter starts on a 64-element
boundary of the flat layout).  State is exposed in torch.optim's ``state_dict`` layout
(exp_avg / exp_avg_sq / momentum_buffer / step per parameter) plus ``master`` (fp32 weights).
"""
from __future__ import annotations

import torch

from .._ext import kernels
from ..parallel.flat import FlatLayout, shared_flat


class _MasterBase(torch.optim.Optimizer):
    _state_keys: tuple = ()

    capturable = False

    def __init__(self, params, defaults, grad_scale: float):
        super().__init__(params, defaults)
        self.grad_scale = grad_scale
        self._flat = None
        self._step = 0
        hp = {tuple((k, tuple(v) if isinstance(v, (list, tuple)) else v) for k, v in g.items()
                    if k not in ("params", "weight_decay")) for g in self.param_groups}
        if len(hp) != 1:
            raise ValueError(f"{type(self).__name__}: hyper-parameters other than weight_decay must be equal "
                             "across groups")

    def _all_params(self):
        return [p for g in self.param_groups for p in g["params"]]

    def _build(self):
        params = self._all_params()
        if not all(p.is_cuda and p.dtype == torch.bfloat16 for p in params):
            raise TypeError(f"{type(self).__name__}: bf16 GPU parameters expected")
        tag = shared_flat(params)
        if tag is None:
            named = {f"p{i}": p for i, p in enumerate(params)}
            layout = FlatLayout([(n, tuple(p.shape)) for n, p in named.items()], [list(named)])
            fp, fg = layout.bind(named, dtype=torch.bfloat16)
        else:
            layout, fp, fg = tag
        n = fp.numel()
        if n % 64:
            raise ValueError("flat buffer must be padded to 64 elements")
        dev = fp.device
        decay = torch.zeros(n // 64, dtype=torch.uint8)
        wd_values = {g["weight_decay"] for g in self.param_groups if g["weight_decay"] != 0.0}
        if len(wd_values) > 1:
            raise ValueError("at most one non-zero weight_decay value across groups")
        self._wd = wd_values.pop() if wd_values else 0.0
        for g in self.param_groups:
            if g["weight_decay"] == 0.0:
                continue
            for p in g["params"]:
                s = layout.slots[p._pde_flat[3]]
                decay[s.offset // 64:(s.offset + s.numel + 63) // 64] = 1
        bufs = {"master": fp.float()}
        for k in self._state_keys:
            bufs[k] = torch.zeros(n, device=dev, dtype=torch.float32)
        self._flat = dict(layout=layout, p=fp, g=fg, bufs=bufs, decay=decay.to(dev),
                          sumsq=torch.zeros(1025, device=dev, dtype=torch.float32),   # [0] + partials
                          step_dev=torch.full((1,), float(self._step), device=dev, dtype=torch.float32))
        for p in params:
            st = self.state[p]
            name = p._pde_flat[3]
            for k, buf in bufs.items():
                st[k] = layout.view(buf, name)
            st["step"] = self._flat["step_dev"] if self.capturable else torch.tensor(float(self._step))

    def state_tensors(self):
        """The optimizer's device state (fp32 master weights, moments, device step count): what a caller
        snapshots and restores around trial steps (``parallel.tune_bucket_cap(restore=...)``), together
        with the host step count ``_step``."""
        if self._flat is None:
            self._build()
        return list(self._flat["bufs"].values()) + [self._flat["step_dev"]]

    def _sync_grads(self):
        f = self._flat
        for p in self._all_params():
            v = f["layout"].view(f["g"], p._pde_flat[3])
            if p.grad is None:
                v.zero_()
                p.grad = v
            elif p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v

    def zero_grad(self, set_to_none: bool = True):
        """Default (torch semantics): gradients become None.  Ops that know the flat layout then write
        the next gradients straight into the flat buffer (``parallel.flat.flat_grad_slot``) and
        ``step`` zero-fills the slots of parameters that received none; ``set_to_none=False`` zeroes
        the flat buffer and keeps the views."""
        if self._flat is not None and not set_to_none:
            self._flat["g"].zero_()
        else:
            for p in self._all_params():
                p.grad = None

    def _kernel(self):  # pragma: no cover - abstract
        raise NotImplementedError

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._flat is None:
            self._build()
        self._sync_grads()
        self._step += 1
        self._kernel()
        if not self.capturable:
            for p in self._all_params():
                self.state[p]["step"] = torch.tensor(float(self._step))
        return loss

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        if self._flat is None:
            self._build()
        f = self._flat
        for p in self._all_params():
            st = self.state[p]
            name = p._pde_flat[3]
            for k, buf in f["bufs"].items():
                view = f["layout"].view(buf, name)
                if k in st and isinstance(st[k], torch.Tensor) and st[k].data_ptr() != view.data_ptr():
                    view.copy_(st[k].to(view.device, view.dtype))
                elif k == "master" and (k not in st or st[k].data_ptr() != view.data_ptr()):
                    view.copy_(p.detach().float())
                st[k] = view
            self._step = int(float(st.get("step", 0)))
        f["step_dev"].fill_(float(self._step))
        if self.capturable:
            for p in self._all_params():
                self.state[p]["step"] = f["step_dev"]
        kernels().f32_to_bf16(f["bufs"]["master"], f["p"])     # the bf16 weights follow the master copy


class AdamWMaster(_MasterBase):
    _state_keys = ("exp_avg", "exp_avg_sq")

    def __init__(self, params, lr=6e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=None,
                 grad_scale: float = 1.0, capturable: bool = False):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay), grad_scale)
        self.max_grad_norm = max_grad_norm
        # capturable (torch.optim's name): the step count is a device tensor read by the kernel, so a
        # step captured into a hipGraph and replayed applies the right bias corrections; the per-param
        # state "step" is then that shared device tensor
        self.capturable = capturable

    def _kernel(self):
        f, K = self._flat, kernels()
        clip = None
        # capturable: the device step count advances in stream order (a graph replay counts too) --
        # inside the grad-norm reduction's one-block finish kernel when clipping, else by an add
        inc = f["step_dev"] if self.capturable else None
        if self.max_grad_norm is not None:
            K.sumsq_bf16(f["g"], self.grad_scale, f["sumsq"], inc)    # deterministic: replicas never drift
            clip = f["sumsq"][:1]
        elif inc is not None:
            inc.add_(1.0)
        g0 = self.param_groups[0]
        b1, b2 = g0["betas"]
        K.adamw_master(f["bufs"]["master"], f["p"], f["g"], f["bufs"]["exp_avg"], f["bufs"]["exp_avg_sq"], g0["lr"],
                       b1, b2, g0["eps"], self._wd, self.grad_scale, self._step, f["decay"], clip,
                       float(self.max_grad_norm or 1.0), f["step_dev"] if self.capturable else None)

    def grad_norm(self) -> float:
        """Global grad norm of the last clipped step (host sync; for logging only)."""
        return float(self._flat["sumsq"][0].sqrt()) if self._flat is not None else 0.0


class SGDMaster(_MasterBase):
    _state_keys = ("momentum_buffer",)

    def __init__(self, params, lr=0.1, momentum=0.9, weight_decay=0.0, nesterov=False, grad_scale: float = 1.0):
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, nesterov=nesterov),
                         grad_scale)

    def _kernel(self):
        f = self._flat
        g0 = self.param_groups[0]
        kernels().sgd_master(f["bufs"]["master"], f["p"], f["g"], f["bufs"]["momentum_buffer"], g0["lr"],
                             g0["momentum"], self._wd, g0["nesterov"], self.grad_scale, f["decay"])
