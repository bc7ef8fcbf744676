"""ResNet-18 bf16 benchmark (``python bench.py --model resnet18``): synthetic 3x224x224 images,
channels-last bf16, DDP over RCCL, fused BN+ReLU kernels, SGD(momentum 0.9, wd 5e-5) with fp32
master weights.  Metric: images/s for the whole node (weak scaling: fixed per-GPU batch)."""
from __future__ import annotations

import json

from bench_models import _cap, _setup, _timed, _tune


def bench_resnet18(args):
    torch, dist, rank, world, dev = _setup()
    from pytorch_distributed_example_amd import ops
    from pytorch_distributed_example_amd.models import build_resnet18
    from pytorch_distributed_example_amd.optim import SGDMaster
    from pytorch_distributed_example_amd.parallel import DistributedDataParallel

    B = args.batch_size if args.batch_size != 128 else 256
    model = build_resnet18(seed=args.seed, device=dev)
    ddp = DistributedDataParallel(model, bucket_cap_mb=_cap(args)) if world > 1 else model
    opt = SGDMaster(model.decay_groups(5e-5), lr=0.1, momentum=0.9)
    # 8 batches per rank of class-conditional synthetic images, sharded by the DistributedSampler
    from pytorch_distributed_example_amd.data import DistributedSampler, synthetic_images
    pool = 8 * B * world
    sampler = DistributedSampler(range(pool), num_replicas=world, rank=rank, shuffle=True, seed=args.seed)
    X, Y = synthetic_images(sampler.indices_tensor().long(), seed=args.seed, device=dev)
    nb = X.shape[0] // B
    it = [0]
    losses = []

    ones = torch.ones((), device=dev, dtype=torch.float32)        # d loss / d loss (no fill kernel per step)

    def eager_step(x, y):
        opt.zero_grad()
        loss = ops.cross_entropy(ddp(x), y)       # bf16 logits straight into the CE kernel (no cast)
        loss.backward(ones)
        opt.step()
        return loss.detach()

    def step():
        i = it[0] % nb
        it[0] += 1
        losses.append(eager_step(X[i * B:(i + 1) * B], Y[i * B:(i + 1) * B]))

    extra = _tune(ddp, step, world, args,
                  restore=list(model.parameters()) + list(model.buffers()) + opt.state_tensors())
    use_graph = args.model_graph == "on" or (args.model_graph == "auto" and world == 1)
    if use_graph:
        # the whole step (forward, loss, backward, SGD with its flat fp32 master / momentum buffers) is
        # captured once into a hipGraph and replayed: ~230 kernel launches per step leave the host, and
        # the ~0.3 ms of launch gaps with them.  Each step copies its batch into the static input first
        # (inside the timed region).  SGDMaster has no host-side step state, so a replay is exact.
        sx, sy = X[:B].clone(), Y[:B].clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):                      # allocator / autograd warm-up outside the capture
                eager_step(sx, sy)
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static_loss = eager_step(sx, sy)

        def step():                                  # noqa: F811 - the graph-replay step
            i = it[0] % nb
            it[0] += 1
            sx.copy_(X[i * B:(i + 1) * B])
            sy.copy_(Y[i * B:(i + 1) * B])
            graph.replay()
            losses.append(static_loss)

        graph.replay()                               # first launch of the graph outside the timed window
        extra["mode"] = "hipgraph (whole step)"
    else:
        extra["mode"] = "eager"
    elapsed = _timed(torch, dist, world, step, args.warmup, args.steps)
    ips = args.steps * B * world / elapsed
    if rank == 0:
        from pytorch_distributed_example_amd.utils.stdio import emit_result
        emit_result({
            "metric": "images/sec (whole node), ResNet-18 bf16 DDP",
            "value": round(ips, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic class-conditional 3x224x224 images (class prototype + noise), 8 batches per rank "
                    "sharded by DistributedSampler, random-init weights",
            "config": {"model": "ResNet-18 (11.69M params, torchvision layout)", "global_batch": B * world,
                       "per_gpu_batch": B, "seq_len": None, "parallelism": f"dp{world}",
                       "optimizer": "SGD(0.1, momentum 0.9, wd 5e-5; fp32 master)", **extra,
                       "memory_format": "channels_last"},
            "last_loss": round(float(losses[-1]), 4),
        })
    if world > 1:
        dist.destroy_process_group()
