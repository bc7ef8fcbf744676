"""Single-node multi-process launcher: one process per GPU (the reference starts every rank by hand in
its own shell -- /root/reference/README.md, mnist/main.py:215-220 -- and pins all of them to GPU 0).

    python -m pytorch_distributed_example_amd.launch --nproc-per-node 8 scripts/mnist.py --epochs 1
    python -m pytorch_distributed_example_amd.launch -n 3 --module some.module -- args

Each child gets ``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``, ``MASTER_ADDR``,
``MASTER_PORT`` (rendezvous ``env://``) and, on ROCm, ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is kept;
with several ranks per node ``OMP_NUM_THREADS`` defaults to cores / ranks (CPU ranks would otherwise
oversubscribe the host nproc-fold).
The launcher never initialises the GPU itself (it only spawns children), monitors them, and on the
first non-zero exit terminates the remaining ranks' process groups (so a failed rank never leaves
its peers hung inside a collective), then exits with that code.  ``--max-restarts`` re-launches the
whole gang (elastic-lite) after a failure.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def _spawn(cmd, env, log_dir, rank, stdout=None):
    out = None
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
        out = open(os.path.join(log_dir, f"rank{rank}.log"), "w")
    # own process group per rank so a kill takes the rank's children with it
    return subprocess.Popen(cmd, env=env, stdout=out or stdout, stderr=subprocess.STDOUT if out else None,
                            start_new_session=True), out


def _terminate(procs, grace: float):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + grace
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def run_gang(cmd, nproc, master_addr, master_port, node_rank=0, nnodes=1, log_dir=None, extra_env=None,
             grace=5.0, poll=0.05, stdout=None):
    """Start ``nproc`` ranks of ``cmd``; returns the first failing exit code (0 if all succeed).
    ``stdout``: where the ranks' stdout goes when there is no ``log_dir`` (default: inherited)."""
    procs, files = [], []
    world = nproc * nnodes
    for local in range(nproc):
        rank = node_rank * nproc + local
        env = dict(os.environ)
        env.update(extra_env or {})
        env.update({"RANK": str(rank), "LOCAL_RANK": str(local), "WORLD_SIZE": str(world),
                    "LOCAL_WORLD_SIZE": str(nproc), "GROUP_RANK": str(node_rank),
                    "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if nproc > 1 and "OMP_NUM_THREADS" not in (extra_env or {}) and "OMP_NUM_THREADS" not in os.environ:
            # CPU ranks share the host: split its cores instead of oversubscribing them nproc-fold
            env["OMP_NUM_THREADS"] = str(max(1, (os.cpu_count() or 1) // nproc))
        p, f = _spawn(cmd, env, log_dir, rank, stdout)
        procs.append(p)
        files.append(f)
    rc = 0
    try:
        alive = set(range(nproc))
        while alive:
            for i in list(alive):
                code = procs[i].poll()
                if code is None:
                    continue
                alive.discard(i)
                if code != 0:
                    sys.stderr.write(f"[launch] rank {node_rank * nproc + i} exited with {code}; "
                                     f"terminating {len(alive)} remaining rank(s)\n")
                    rc = code if code > 0 else 128 - code
                    _terminate(procs, grace)
                    alive.clear()
                    break
            time.sleep(poll)
    except KeyboardInterrupt:
        _terminate(procs, grace)
        rc = 130
    finally:
        for f in files:
            if f:
                f.close()
    return rc


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--nproc-per-node", "-n", type=int, default=1)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node-rank", type=int, default=0)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=0, help="0 = pick a free port")
    ap.add_argument("--log-dir", default=None, help="write rank<i>.log files instead of inheriting stdio")
    ap.add_argument("--max-restarts", type=int, default=0)
    ap.add_argument("--module", "-m", action="store_true", help="run the target as `python -m module`")
    ap.add_argument("script")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    args = a.script_args[1:] if a.script_args[:1] == ["--"] else a.script_args
    cmd = [sys.executable] + (["-m", a.script] if a.module else [a.script]) + args
    port = a.master_port or free_port(a.master_addr)
    rc = 0
    for attempt in range(a.max_restarts + 1):
        rc = run_gang(cmd, a.nproc_per_node, a.master_addr, port, a.node_rank, a.nnodes, a.log_dir,
                      extra_env={"PDE_RESTART_COUNT": str(attempt)})
        if rc == 0:
            break
        if attempt < a.max_restarts:
            sys.stderr.write(f"[launch] restarting gang (attempt {attempt + 2}/{a.max_restarts + 1})\n")
            if not a.master_port:
                port = free_port(a.master_addr)
    return rc


if __name__ == "__main__":
    sys.exit(main())
