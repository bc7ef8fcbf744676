"""Helper: run ``tests/mp_workers.py <case>`` on W local ranks through the framework launcher."""
from __future__ import annotations

import json
import os
import sys
import tempfile

from pytorch_distributed_example_amd.launch import free_port, run_gang

HERE = os.path.dirname(os.path.abspath(__file__))


def run_ranks(case, world, *args, timeout_env=None, extra_env=None):
    with tempfile.TemporaryDirectory() as d:
        cmd = [sys.executable, os.path.join(HERE, "mp_workers.py"), case, *map(str, args)]
        env = {"PYTHONWARNINGS": "ignore::FutureWarning"}
        env.update(extra_env or {})
        rc = run_gang(cmd, world, "127.0.0.1", free_port(), log_dir=d, extra_env=env)
        logs = []
        for r in range(world):
            with open(os.path.join(d, f"rank{r}.log")) as f:
                logs.append(f.read())
    results = []
    for log in logs:
        res = [json.loads(l[len("RESULT "):]) for l in log.splitlines() if l.startswith("RESULT ")]
        results.append(res[-1] if res else None)
    return rc, results, logs
