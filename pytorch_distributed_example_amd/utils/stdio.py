"""fd-level stdout redirection.

RCCL prints a version banner ("RCCL version : ...", "HIP version", ...) on the process's stdout
when a communicator is created.  Benchmarks whose stdout contract is ONE JSON line wrap process-group
setup in ``stdout_to_stderr()`` so such native chatter lands on stderr instead.  libc's own stdout
buffer is flushed before fd 1 is restored, so nothing written meanwhile leaks out later.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import sys


def _c_fflush():
    try:
        ctypes.CDLL(None).fflush(None)
    except Exception:   # noqa: BLE001 - best effort
        pass


@contextlib.contextmanager
def stdout_to_stderr():
    sys.stdout.flush()
    _c_fflush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        _c_fflush()
        os.dup2(saved, 1)
        os.close(saved)


def emit_result(obj) -> None:
    """Print a benchmark's one JSON result line (rank 0).  Under ``bench.py``'s self-launch
    (``PDE_BENCH_RESULT`` names a file) the line is also written there: the ranks' stdout goes to the
    parent's stderr, and the parent relays exactly this line on its own stdout."""
    import json

    line = json.dumps(obj)
    print(line, flush=True)
    path = os.environ.get("PDE_BENCH_RESULT")
    if path:
        with open(path, "w") as f:
            f.write(line + "\n")
