#!/usr/bin/env python3
"""Collective smoke test with the reference's flags and output (/root/reference/toy/main.py).

Every rank draws an integer in [0, 10] per step and all-reduces it (SUM) over a group holding all
ranks, then prints ``rank: R, step: S, value: V, reduced sum: X.``.  The reference builds that group
anew each step (toy/main.py:16).  ``dist.new_group`` here returns the communicator cached for the
rank tuple, so the per-step rebuild costs nothing.

  python3 scripts/toy.py -i tcp://127.0.0.1:23456 -r 0 -s 3     (one shell per rank, as the reference)
  python3 -m pytorch_distributed_example_amd.launch --nproc-per-node 3 scripts/toy.py
"""
import argparse
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_example_amd import dist  # noqa: E402

# (flags, argparse keywords): names, defaults and dest order as toy/main.py:34-56 (the Namespace line
# printed at start-up lists them in this order); --sleep is additive (the reference pauses 1 s)
_FLAGS = (
    (("--backend",), dict(type=str, default="gloo", help="Name of the backend to use.")),
    (("--init-method", "-i"), dict(type=str, default="tcp://127.0.0.1:23456",
                                    help="URL specifying how to initialize the package.")),
    (("--rank", "-r"), dict(type=int, help="Rank of the current process.")),
    (("--world-size", "-s"), dict(type=int, help="Number of processes participating in the job.")),
    (("--steps",), dict(type=int, default=20)),
    (("--sleep",), dict(type=float, default=1.0, help="Pause per step in seconds.")),
)


def _reduce_step(world_size: int) -> tuple:
    """One step: this rank's draw and the SUM over every rank (a group spanning them all)."""
    drawn = random.randint(0, 10)
    everyone = dist.new_group(ranks=list(range(world_size)))
    buf = torch.IntTensor([drawn])
    dist.all_reduce(buf, op=dist.reduce_op.SUM, group=everyone)
    return drawn, float(buf)


def foo(rank, world_size, steps, pause=1.0):
    """The reference's loop (toy/main.py:9-25): ``steps`` all-reduces, one output line each."""
    step = 0
    while step < steps:
        step += 1
        drawn, total = _reduce_step(world_size)
        print(f"rank: {rank}, step: {step}, value: {drawn}, reduced sum: {total}.", flush=True)
        time.sleep(pause)


def init_process(backend, init_method, rank, world_size):
    """Join the process group (toy/main.py:28-33)."""
    dist.init_process_group(backend=backend, init_method=init_method, rank=rank, world_size=world_size)


def _parse(argv):
    parser = argparse.ArgumentParser()
    for names, kw in _FLAGS:
        parser.add_argument(*names, **kw)
    args = parser.parse_args(argv)
    # launcher mode (torchrun / our launch.py): rank and world size from the environment when not given
    if args.rank is None and "RANK" in os.environ:
        args.rank = int(os.environ["RANK"])
        args.init_method = "env://"
    if args.world_size is None and "WORLD_SIZE" in os.environ:
        args.world_size = int(os.environ["WORLD_SIZE"])
    return args


def main(argv=None):
    args = _parse(argv)
    print(args, flush=True)
    init_process(args.backend, args.init_method, args.rank, args.world_size)
    foo(args.rank, args.world_size, args.steps, args.sleep)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
