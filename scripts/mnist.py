#!/usr/bin/env python3
"""Data-parallel CNN trainer with the reference's flags and output (/root/reference/mnist/main.py).

Reference flags/defaults are kept (--backend nccl, -i/--init-method tcp://127.0.0.1:23456, -r, -s,
--epochs 20, --no-cuda, -lr 1e-3, --root data, --batch-size 128, --eval) and so is the printed
sequence (Namespace, "called init_process_group", "device = ...", "Getting data loader with root =
...", "obtained data_loader", "Epoch: e/E, train loss: ..., train acc: ..%, test loss: ..., test
acc: ..%.").  Fixed reference defects: the :211 syntax error, unsynchronised replicas (seeded init +
rank-0 broadcast), every local rank on GPU 0 (one GPU per local rank).  Kept quirks: train set
"FashionMNIST", test set "MNIST" (two independent synthetic sets here -- no network), no
``set_epoch`` unless --set-epoch, ``-s 1`` skips the process group.

Additive flags: --engine {auto,fused,autograd}, --ddp {on,off} (off = the reference's per-parameter
``average_gradients``), --model {net,mlp}, --optimizer {adam,sgd}, --seed, --train-size,
--test-size, --save/--resume (state_dict compatible), --cprofile PATH (default ./stats, like the
reference's always-on cProfile wrapper; --no-cprofile turns it off), --metrics PATH (JSONL),
--log-rank0-only, --no-graph, --set-epoch, --bucket-mb (DDP gradient bucket cap, autograd engine),
--dtype {fp32,bf16} (bf16: torch.autocast mixed precision over the ATen layer path with fp32
parameters, gradients and optimizer state; the fused engine and the framework's toy-CNN kernels are
fp32, the reference's dtype).
"""
import argparse
import cProfile
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_example_amd import dist  # noqa: E402
from pytorch_distributed_example_amd.data import (DeviceDataLoader, DistributedSampler, RandomSampler,  # noqa: E402
                                                  idx_dataset, synthetic_mnist)
from pytorch_distributed_example_amd.engine import LeNetTrainStep  # noqa: E402
from pytorch_distributed_example_amd.engine.trainer import FusedTrainer, Trainer  # noqa: E402
from pytorch_distributed_example_amd.models import MLP, build_net  # noqa: E402
from pytorch_distributed_example_amd.optim import SGD, Adam  # noqa: E402
from pytorch_distributed_example_amd.parallel import DistributedDataParallel  # noqa: E402
from pytorch_distributed_example_amd.utils.checkpoint import load_checkpoint, save_checkpoint  # noqa: E402


def get_datasets(root, device, train_size, test_size, seed):
    train = idx_dataset(os.path.join(root, "FashionMNIST", "raw"), True, device)
    if train is None:
        train = synthetic_mnist(train_size, seed=seed, device=device, kind="fashion")
    test = idx_dataset(os.path.join(root, "MNIST", "raw"), False, device)
    if test is None:
        test = synthetic_mnist(test_size, seed=seed, device=device, kind="digits")
    return train, test


def get_dataloader(root, batch_size, world_size, device="cpu", train_size=60000, test_size=10000, seed=0):
    print("Getting data loader with root = {}".format(root))
    train_set, test_set = get_datasets(root, device, train_size, test_size, seed)
    if world_size == 1:
        train_loader = DeviceDataLoader(train_set, batch_size=batch_size, shuffle=True, seed=seed)
    else:
        sampler = DistributedSampler(train_set)
        train_loader = DeviceDataLoader(train_set, batch_size=batch_size, shuffle=(sampler is None), sampler=sampler)
    test_loader = DeviceDataLoader(test_set, batch_size=batch_size, shuffle=False)
    return train_loader, test_loader


def pick_device(args):
    if torch.cuda.is_available() and not args.no_cuda:
        n = torch.cuda.device_count()
        local = int(os.environ.get("LOCAL_RANK", (args.rank or 0) % max(1, n)))
        torch.cuda.set_device(local)
        return torch.device("cuda", local)
    return torch.device("cpu")


class _Printer:
    def __init__(self, enabled, metrics_path, images_per_epoch):
        self.enabled = enabled
        self.metrics = open(metrics_path, "a") if metrics_path else None
        self.t0 = time.perf_counter()
        self.images = images_per_epoch

    def __call__(self, *parts):
        if self.enabled:
            print(*parts, flush=True)
        if self.metrics is not None:
            now = time.perf_counter()
            line = " ".join(parts)
            self.metrics.write(json.dumps({"line": line, "epoch_time_s": now - self.t0,
                                           "images_per_s": self.images / max(1e-9, now - self.t0)}) + "\n")
            self.metrics.flush()
            self.t0 = now


def run(args):
    device = pick_device(args)
    print("device = {}".format(device.type))
    world = args.world_size if args.world_size is not None else 1
    rank = dist.get_rank() if dist.is_initialized() else 0

    if args.model == "mlp":
        torch.manual_seed(args.seed)
        net = MLP().to(device)
    else:
        net = build_net(seed=args.seed, device=device)

    train_loader, test_loader = get_dataloader(args.root, args.batch_size, world, device, args.train_size,
                                               args.test_size, args.seed)
    print("obtained data_loader")

    distributed = False if world == 1 else True
    engine = args.engine
    if args.dtype == "bf16":
        if engine == "fused":
            raise SystemExit("--dtype bf16 needs --engine autograd (the fused toy-CNN engine is fp32)")
        engine = "autograd"
        net.aten = True                  # the layer path through torch.nn.functional, autocast to bf16
    if engine == "auto":
        engine = "fused" if (device.type == "cuda" and args.model == "net" and
                             (not distributed or dist.get_backend() in ("nccl", "rccl"))) else "autograd"
    printer = _Printer(not args.log_rank0_only or rank == 0, args.metrics if rank == 0 else None,
                       len(train_loader.sampler) * max(1, world))

    if distributed:
        dist.broadcast_parameters(net)          # fixes survey Q2: replicas start identical
    start_epoch = 0
    payload = None
    if args.resume:
        payload = load_checkpoint(args.resume, net)
        start_epoch = int(payload.get("epoch", 0))

    if engine == "fused":
        comm = dist.engine_comm() if distributed else None
        eng = LeNetTrainStep(net, batch_size=args.batch_size, lr=args.learning_rate, optimizer=args.optimizer,
                             comm=comm)
        if payload is not None and "optimizer" in payload:
            eng.load_optimizer_state_dict(payload["optimizer"])
        eng.sync_params()
        trainer = FusedTrainer(eng, train_loader.dataset, test_loader.dataset, train_loader.sampler, args.eval,
                               use_graph=not args.no_graph, set_epoch=args.set_epoch)
        opt_state = eng.optimizer_state_dict
    else:
        model = net
        if distributed and args.ddp == "on":
            model = DistributedDataParallel(net, init_sync=False, bucket_cap_mb=args.bucket_mb)
        params = model.parameters()
        optimizer = (Adam(params, lr=args.learning_rate) if args.optimizer == "adam"
                     else SGD(params, lr=args.learning_rate, momentum=0.9))
        if payload is not None and "optimizer" in payload:
            optimizer.load_state_dict(payload["optimizer"])
        trainer = Trainer(model, optimizer, train_loader, test_loader, device, distributed, args.eval,
                          manual_average=(args.ddp == "off"),
                          autocast_dtype=torch.bfloat16 if args.dtype == "bf16" else None)
        trainer.set_epoch = args.set_epoch
        opt_state = optimizer.state_dict
    trainer.printer = printer

    epochs = args.epochs
    # resume: epochs start_epoch+1..E, numbered (and --set-epoch seeded) as in an uninterrupted run
    trainer.fit(epochs, start_epoch=start_epoch)
    if engine == "fused":
        trainer.check_comm_health()        # never checkpoint replicas a failed all-reduce let diverge
    if args.save:
        save_checkpoint(args.save, net, opt_state(), epoch=epochs, rank=rank)


def init_process(args):
    dist.init_process_group(
        backend=args.backend,
        init_method=args.init_method,
        rank=args.rank,
        world_size=args.world_size)
    print("called init_process_group")


def build_parser():
    parser = argparse.ArgumentParser()
    parser.add_argument('--backend', type=str, default='nccl', help='Name of the backend to use.')
    parser.add_argument('-i', '--init-method', type=str, default='tcp://127.0.0.1:23456',
                        help='URL specifying how to initialize the package.')
    parser.add_argument('-r', '--rank', type=int, help='Rank of the current process.')
    parser.add_argument('-s', '--world-size', type=int, help='Number of processes participating in the job.')
    parser.add_argument('--epochs', type=int, default=20)
    parser.add_argument('--no-cuda', action='store_true')
    parser.add_argument('--learning-rate', '-lr', type=float, default=1e-3)
    parser.add_argument('--root', type=str, default='data')
    parser.add_argument('--batch-size', type=int, default=128)
    parser.add_argument('--eval', action='store_true', default=False)
    # additive flags
    parser.add_argument('--engine', choices=['auto', 'fused', 'autograd'], default='auto')
    parser.add_argument('--ddp', choices=['on', 'off'], default='on')
    parser.add_argument('--model', choices=['net', 'mlp'], default='net')
    parser.add_argument('--optimizer', choices=['adam', 'sgd'], default='adam')
    parser.add_argument('--seed', type=int, default=0)
    parser.add_argument('--train-size', type=int, default=60000)
    parser.add_argument('--test-size', type=int, default=10000)
    parser.add_argument('--save', type=str, default=None)
    parser.add_argument('--resume', type=str, default=None)
    parser.add_argument('--cprofile', type=str, default='stats',
                        help="pstats file of the whole run (reference: cProfile.run('main()', 'stats'), always on); "
                             "rank-suffixed when several ranks share a directory")
    parser.add_argument('--no-cprofile', action='store_true', help='run without the cProfile wrapper')
    parser.add_argument('--metrics', type=str, default=None, help='append per-epoch JSONL metrics (rank 0)')
    parser.add_argument('--log-rank0-only', action='store_true')
    parser.add_argument('--no-graph', action='store_true', help='fused engine: launch eagerly (no hipGraph)')
    parser.add_argument('--set-epoch', action='store_true', help='reshuffle shards every epoch')
    parser.add_argument('--bucket-mb', type=float, default=25.0,
                        help='DDP gradient bucket cap in MB (autograd engine; the fused engine times its '
                             'own one- / two-bucket schedules)')
    parser.add_argument('--dtype', choices=['fp32', 'bf16'], default='fp32',
                        help='compute dtype: bf16 = autocast mixed precision (fp32 params / grads / Adam state)')
    return parser


def main(argv=None):
    args = build_parser().parse_args(argv)
    # launcher mode (torchrun / pytorch_distributed_example_amd.launch): env:// rendezvous
    if args.rank is None and "RANK" in os.environ:
        args.rank = int(os.environ["RANK"])
        args.world_size = int(os.environ["WORLD_SIZE"])
        args.init_method = "env://"
    print(args)

    if (args.world_size != 1):
        init_process(args)
    run(args)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == '__main__':
    argv = sys.argv[1:]
    # like the reference (main.py:241-242) every run is profiled into ./stats unless --no-cprofile
    if '--no-cprofile' not in argv and '-h' not in argv and '--help' not in argv:
        path = argv[argv.index('--cprofile') + 1] if '--cprofile' in argv else 'stats'
        rank = os.environ.get("RANK")
        if '-r' in argv or '--rank' in argv:
            k = argv.index('-r') if '-r' in argv else argv.index('--rank')
            rank = argv[k + 1]
        multi = os.environ.get("WORLD_SIZE", "1") != "1"
        for flag in ('-s', '--world-size'):
            if flag in argv:
                multi = argv[argv.index(flag) + 1] != '1'
        if rank is not None and multi:
            path = f"{path}.rank{rank}"
        cProfile.run('main()', path)
    else:
        main()
