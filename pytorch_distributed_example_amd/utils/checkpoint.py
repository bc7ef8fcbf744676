"""Checkpoint / resume, state_dict-compatible with the reference model and torch.optim.Adam.

The reference has no checkpointing (survey §5).  We add it without changing formats: the model
part is exactly ``Net().state_dict()`` of /root/reference/mnist/main.py:130-137 (keys
``conv1.weight`` … ``fc2.bias``, fp32, CPU tensors), the optimizer part is
``torch.optim.Adam.state_dict()`` layout.  Rank 0 writes; every rank loads with
``torch.load(weights_only=True)`` (no pickle code execution) and, when distributed, rank 0's copy is
broadcast so all replicas restart identical.
"""
from __future__ import annotations

import os

import torch


def _cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().to("cpu").clone()
    if isinstance(obj, dict):
        return {k: _cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu(v) for v in obj)
    return obj


def unwrap(model):
    return getattr(model, "module", model)


def save_checkpoint(path: str, model, optimizer_state=None, epoch: int = 0, extra=None, rank: int = 0):
    if rank != 0:
        return
    payload = {"model": _cpu(unwrap(model).state_dict()), "epoch": int(epoch)}
    if optimizer_state is not None:
        payload["optimizer"] = _cpu(optimizer_state)
    if extra:
        payload["extra"] = _cpu(extra)
    tmp = path + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save(payload, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str, model, map_location="cpu", broadcast: bool = True):
    """Load into ``model`` (in place); returns the payload (optimizer state, epoch, ...)."""
    payload = torch.load(path, map_location=map_location, weights_only=True)
    sd = payload["model"] if "model" in payload else payload      # a bare state_dict also works
    unwrap(model).load_state_dict(sd)
    if broadcast:
        from .. import dist

        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.broadcast_parameters(unwrap(model))
    return payload
