"""Loader for the in-tree native extension modules (``_lib/_kernels*.so``, ``_lib/_runtime*.so``).

The shared objects are built by :mod:`pytorch_distributed_example_amd.utils.build` (explicit hipcc
for gfx950) and live inside the package directory so they travel with the repo snapshot.  There
is deliberately NO silent fallback: GPU code paths call :func:`kernels`, which raises if the HIP
extension is missing or failed to load, so a run can never quietly use stock ATen ops instead.
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import sys
import threading

_LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
_lock = threading.Lock()
_cache: dict = {}


class NativeExtensionError(RuntimeError):
    pass


def _so_path(name: str) -> str:
    for suf in importlib.machinery.EXTENSION_SUFFIXES:
        p = os.path.join(_LIBDIR, name + suf)
        if os.path.exists(p):
            return p
    return ""


def _load(name: str, auto_build: bool):
    with _lock:
        if name in _cache:
            return _cache[name]
        import torch  # noqa: F401  -- load torch's libamdhip64 / librccl first (same sonames)

        path = _so_path(name)
        if not path and auto_build and os.environ.get("PDE_NO_AUTOBUILD") != "1":
            from .utils.build import build

            build([name])
            path = _so_path(name)
        if not path:
            raise NativeExtensionError(
                f"native extension {name} not built (expected under {_LIBDIR}); run "
                f"`python -m pytorch_distributed_example_amd.utils.build`")
        modname = f"pytorch_distributed_example_amd._lib.{name}"
        spec = importlib.util.spec_from_file_location(modname, path)
        if spec is None or spec.loader is None:
            raise NativeExtensionError(f"cannot load {path}")
        mod = importlib.util.module_from_spec(spec)
        try:
            spec.loader.exec_module(mod)
        except ImportError as e:  # pragma: no cover - surfaced loudly
            raise NativeExtensionError(f"failed to load {path}: {e}") from e
        sys.modules[modname] = mod
        _cache[name] = mod
        return mod


def kernels(auto_build: bool = True):
    """The HIP kernel module (raises NativeExtensionError if unavailable)."""
    return _load("_kernels", auto_build)


def runtime(auto_build: bool = True):
    """The C++ distributed runtime module (store, host collectives, RCCL communicator)."""
    return _load("_runtime", auto_build)


def loaded_native_libraries() -> list:
    """Paths of the in-tree shared objects loaded in this process (for reports / smoke checks)."""
    return sorted(getattr(m, "__file__", "") for m in _cache.values())
