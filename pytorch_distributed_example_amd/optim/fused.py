"""Fused Adam / AdamW / SGD: one HIP launch per parameter group per step (csrc/kernels/optim.hip).

The reference builds ``torch.optim.Adam(net.parameters(), lr)`` (/root/reference/mnist/main.py:187)
whose CUDA default is a multi-tensor ``foreach`` chain of ~8 launches per step.  Here all
parameters of a group live in one flat fp32 buffer (shared with DDP's gradient buckets when the
model is wrapped first, see ``parallel.flat``), and the whole update is a single fused kernel with
the step counter on the device (capturable in hipGraphs).

The classes subclass ``torch.optim.Optimizer`` so ``state_dict()`` / ``load_state_dict()`` keep
torch's format (``state[i] = {step, exp_avg, exp_avg_sq}`` / ``{momentum_buffer}``): per-parameter
state entries are views into the flat buffers.  CPU parameters (the reference's ``--no-cuda``
path) use the same math with ATen CPU ops.
"""
from __future__ import annotations

import math

import torch

from .._ext import kernels
from ..parallel.flat import FlatLayout, shared_flat


class _FlatGroup:
    def __init__(self, params, state_keys):
        tag = shared_flat(params)
        if tag is None:
            named = {f"p{i}": p for i, p in enumerate(params)}
            layout = FlatLayout([(n, tuple(p.shape)) for n, p in named.items()], [list(named)])
            fp, fg = layout.bind(named)
        else:
            layout, fp, fg = tag
        self.layout, self.params, self.grads = layout, fp, fg
        self.names = [p._pde_flat[3] for p in params]
        self.bufs = {k: torch.zeros_like(fp) for k in state_keys}
        self.step_ctr = torch.zeros(1, device=fp.device, dtype=torch.int64)
        self.arrive = torch.zeros(1, device=fp.device, dtype=torch.int32)
        self.steps = 0

    def view(self, key, p):
        return self.layout.view(self.bufs[key], p._pde_flat[3])

    def sync_grads(self, params):
        """Make every p.grad the flat view (autograd may have replaced it after zero_grad(set_to_none)).

        Returns the parameters whose grad was None: torch.optim skips those, so the caller saves their
        value and state around the fused launch (``_Frozen``) instead of letting the flat kernel move them."""
        missing = []
        for p in params:
            v = self.layout.view(self.grads, p._pde_flat[3])
            if p.grad is None:
                missing.append(p)
                v.zero_()
            elif p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v
        return missing


class _Frozen:
    """Parameters without a gradient this step keep their value and optimizer state, as in torch.optim
    (the flat kernel updates every element; the rare grad-None case restores the saved slices after it).
    The device step counter is shared by the group, so such a parameter's later bias correction uses the
    group's step count rather than a private one."""

    def __init__(self, fg, params):
        self.saved = [(p, p.detach().clone(), {k: fg.view(k, p).clone() for k in fg.bufs}) for p in params]
        self.fg = fg

    def restore(self):
        for p, val, st in self.saved:
            p.data.copy_(val)
            for k, v in st.items():
                self.fg.view(k, p).copy_(v)


class _FusedBase(torch.optim.Optimizer):
    _state_keys = ()

    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self._flat = {}

    def _gpu_group(self, group) -> bool:
        ps = group["params"]
        return bool(ps) and all(p.is_cuda and p.dtype == torch.float32 for p in ps)

    def _prepare(self, gi, group):
        fg = self._flat.get(gi)
        if fg is None:
            fg = _FlatGroup(group["params"], self._state_keys)
            self._flat[gi] = fg
            for p in group["params"]:
                st = self.state[p]
                for k in self._state_keys:
                    if k in st and isinstance(st[k], torch.Tensor):
                        fg.view(k, p).copy_(st[k])
                    st[k] = fg.view(k, p)
                st.setdefault("step", torch.tensor(0.0))
                fg.steps = int(float(st["step"]))
            fg.step_ctr.fill_(fg.steps)
        return fg

    def zero_grad(self, set_to_none: bool = False):
        # default False: keep the flat-buffer views (set_to_none would force a re-bind copy each step)
        for gi, group in enumerate(self.param_groups):
            if gi in self._flat:
                self._flat[gi].grads.zero_()
                if set_to_none:     # torch semantics: grad None until backward writes one (re-bound in step)
                    for p in group["params"]:
                        p.grad = None
                continue
            for p in group["params"]:
                if p.grad is None:
                    continue
                if set_to_none:
                    p.grad = None
                else:
                    if p.grad.grad_fn is not None:
                        p.grad.detach_()
                    else:
                        p.grad.requires_grad_(False)   # DDP bucket views cannot be detached in place
                    p.grad.zero_()

    def _after_step(self, gi, group):
        fg = self._flat[gi]
        fg.steps += 1
        for p in group["params"]:
            self.state[p]["step"] = torch.tensor(float(fg.steps))

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for gi, fg in list(self._flat.items()):
            group = self.param_groups[gi]
            for p in group["params"]:
                st = self.state[p]
                for k in self._state_keys:
                    if k in st and isinstance(st[k], torch.Tensor):
                        fg.view(k, p).copy_(st[k].to(fg.params.device))
                    st[k] = fg.view(k, p)
                fg.steps = int(float(st.get("step", 0)))
            fg.step_ctr.fill_(fg.steps)


class Adam(_FusedBase):
    _state_keys = ("exp_avg", "exp_avg_sq")

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 decoupled_weight_decay=False, grad_scale: float = 1.0):
        if amsgrad:
            raise NotImplementedError("amsgrad")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=True,
                        decoupled_weight_decay=decoupled_weight_decay)
        super().__init__(params, defaults)
        self.grad_scale = grad_scale

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            if self._gpu_group(group):
                fg = self._prepare(gi, group)
                frozen = _Frozen(fg, missing) if (missing := fg.sync_grads(group["params"])) else None
                kernels().adam_flat(fg.params, fg.grads, fg.bufs["exp_avg"], fg.bufs["exp_avg_sq"], group["lr"], b1,
                                    b2, group["eps"], group["weight_decay"], group["decoupled_weight_decay"],
                                    self.grad_scale, fg.step_ctr, fg.arrive, 1)
                if frozen is not None:
                    frozen.restore()
                self._after_step(gi, group)
            else:
                _adam_cpu(self, group, b1, b2)
        return loss


class AdamW(Adam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False):
        super().__init__(params, lr, betas, eps, weight_decay, amsgrad, decoupled_weight_decay=True)


class SGD(_FusedBase):
    _state_keys = ("momentum_buffer",)

    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
                 grad_scale: float = 1.0):
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay, nesterov=nesterov,
                        maximize=False, foreach=None, differentiable=False, fused=True)
        super().__init__(params, defaults)
        self.grad_scale = grad_scale

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            if self._gpu_group(group):
                fg = self._prepare(gi, group)
                frozen = _Frozen(fg, missing) if (missing := fg.sync_grads(group["params"])) else None
                kernels().sgd_flat(fg.params, fg.grads, fg.bufs["momentum_buffer"], group["lr"], group["momentum"],
                                   group["dampening"], group["weight_decay"], group["nesterov"], self.grad_scale,
                                   fg.step_ctr, fg.arrive, 1)
                if frozen is not None:
                    frozen.restore()
                self._after_step(gi, group)
            else:
                _sgd_cpu(self, group)
        return loss


# ---------------------------------------------------------------------------------------------- CPU
def _adam_cpu(opt, group, b1, b2):
    """torch.optim.Adam single-tensor algorithm (torch/optim/adam.py) for CPU parameters."""
    for p in group["params"]:
        if p.grad is None:
            continue
        g = p.grad * opt.grad_scale
        st = opt.state[p]
        if "exp_avg" not in st or not isinstance(st.get("exp_avg"), torch.Tensor):
            st["step"] = torch.tensor(0.0)
            st["exp_avg"] = torch.zeros_like(p)
            st["exp_avg_sq"] = torch.zeros_like(p)
        st["step"] += 1
        t = float(st["step"])
        wd = group["weight_decay"]
        if wd:
            if group.get("decoupled_weight_decay"):
                p.mul_(1 - group["lr"] * wd)
            else:
                g = g.add(p, alpha=wd)
        st["exp_avg"].lerp_(g, 1 - b1)
        st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
        step_size = group["lr"] / (1 - b1 ** t)
        denom = (st["exp_avg_sq"].sqrt() / math.sqrt(1 - b2 ** t)).add_(group["eps"])
        p.addcdiv_(st["exp_avg"], denom, value=-step_size)


def _sgd_cpu(opt, group):
    for p in group["params"]:
        if p.grad is None:
            continue
        d = p.grad * opt.grad_scale
        if group["weight_decay"]:
            d = d.add(p, alpha=group["weight_decay"])
        st = opt.state[p]
        if group["momentum"]:
            buf = st.get("momentum_buffer")
            if buf is None:
                buf = st["momentum_buffer"] = d.clone()
            else:
                buf.mul_(group["momentum"]).add_(d, alpha=1 - group["dampening"])
            d = d.add(buf, alpha=group["momentum"]) if group["nesterov"] else buf
        p.add_(d, alpha=-group["lr"])
