"""Profiling hooks: roctx ranges (visible in rocprofv3 --marker-trace / rocprof-sys timelines),
host cProfile helpers, and a tiny CUDA-event step timer.

``range("name")`` is a context manager that pushes / pops a roctx range through ``libroctx64.so``
(ctypes, no build step); when the library is absent or ``PDE_ROCTX=0`` it is a no-op, so the calls
can stay in the hot loop.  Ranges are host-side annotations: they are NOT recorded inside hipGraph
capture (the captured kernels themselves show up in --kernel-trace).
"""
from __future__ import annotations

import contextlib
import ctypes
import ctypes.util
import os
import time

_ROCTX = None
_ENABLED = os.environ.get("PDE_ROCTX", "1") != "0"


def _lib():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so", ctypes.util.find_library("roctx64")):
            if not name:
                continue
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _ROCTX = lib
                break
            except OSError:
                continue
    return _ROCTX


def available() -> bool:
    return bool(_ENABLED and _lib())


def push(name: str):
    lib = _lib() if _ENABLED else None
    if lib:
        lib.roctxRangePushA(name.encode())


def pop():
    lib = _lib() if _ENABLED else None
    if lib:
        lib.roctxRangePop()


def mark(name: str):
    lib = _lib() if _ENABLED else None
    if lib:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors torch.cuda.nvtx.range
    push(name)
    try:
        yield
    finally:
        pop()


class StepTimer:
    """GPU step timing with device events (no host sync until ``summary()``)."""

    def __init__(self):
        import torch

        self._torch = torch
        self.events = []

    def start(self):
        e = self._torch.cuda.Event(enable_timing=True)
        e.record()
        self.events.append([e, None])

    def stop(self):
        e = self._torch.cuda.Event(enable_timing=True)
        e.record()
        self.events[-1][1] = e

    def summary(self):
        self._torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in self.events if b is not None)
        if not ms:
            return {}
        return {"steps": len(ms), "median_ms": ms[len(ms) // 2], "min_ms": ms[0], "max_ms": ms[-1]}


def cprofile_path(base: str, rank: int | None, world: int) -> str:
    """Rank-suffixed pstats path (the reference writes one unsuffixed ``stats`` per rank, which
    ranks sharing a working directory overwrite -- survey R17)."""
    return base if (rank is None or world <= 1) else f"{base}.rank{rank}"


class WallTimer(contextlib.ContextDecorator):
    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.elapsed = time.perf_counter() - self.t0
        return False
