#!/usr/bin/env python3
"""Collective smoke test with the reference's flags and output (/root/reference/toy/main.py).

Each rank draws a random int per step and all-reduces it (SUM) over a group of all ranks
(recreated every step, exactly like the reference's ``new_group`` at toy/main.py:16 -- our
``new_group`` caches the communicator per rank tuple, so the per-step cost disappears), printing
``rank: R, step: S, value: V, reduced sum: X.``.

  python3 scripts/toy.py -i tcp://127.0.0.1:23456 -r 0 -s 3     (one shell per rank, as the reference)
  python3 -m pytorch_distributed_example_amd.launch --nproc-per-node 3 scripts/toy.py
"""
import argparse
import os
import sys
from random import randint
from time import sleep

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_example_amd import dist  # noqa: E402


def foo(rank, world_size, steps, pause=1.0):
    for step in range(1, steps + 1):
        # get random int
        value = randint(0, 10)

        # group all ranks
        ranks = list(range(world_size))
        group = dist.new_group(ranks=ranks)

        # compute reduced sum
        tensor = torch.IntTensor([value])
        dist.all_reduce(tensor, op=dist.reduce_op.SUM, group=group)

        print('rank: {}, step: {}, value: {}, reduced sum: {}.'.format(
            rank, step, value, float(tensor)), flush=True)

        sleep(pause)


def init_process(backend, init_method, rank, world_size):
    dist.init_process_group(
        backend=backend,
        init_method=init_method,
        rank=rank,
        world_size=world_size)


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument('--backend', type=str, default='gloo', help='Name of the backend to use.')
    parser.add_argument('--init-method', '-i', type=str, default='tcp://127.0.0.1:23456',
                        help='URL specifying how to initialize the package.')
    parser.add_argument('--rank', '-r', type=int, help='Rank of the current process.')
    parser.add_argument('--world-size', '-s', type=int, help='Number of processes participating in the job.')
    parser.add_argument('--steps', type=int, default=20)
    # additive flag: the reference sleeps 1 s per step (toy/main.py:25)
    parser.add_argument('--sleep', type=float, default=1.0, help='Pause per step in seconds.')
    args = parser.parse_args(argv)
    print(args, flush=True)

    # launcher mode: take rank / world size from the environment when not given
    if args.rank is None and "RANK" in os.environ:
        args.rank = int(os.environ["RANK"])
        args.init_method = "env://"
    if args.world_size is None and "WORLD_SIZE" in os.environ:
        args.world_size = int(os.environ["WORLD_SIZE"])
    init_process(args.backend, args.init_method, args.rank, args.world_size)
    foo(args.rank, args.world_size, args.steps, args.sleep)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
