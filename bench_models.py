#!/usr/bin/env python3
"""Benchmarks of the driver-added configs (BASELINE.json ``configs``), same timing contract as
``bench.py`` (W untimed warm-up steps, K timed steps between barrier + synchronize, max over ranks,
one JSON line from rank 0):

* ``--model gpt2``     GPT-2 small (124M), bf16, DDP over RCCL with large gradient buckets,
                       fused AdamW (fp32 master), synthetic tokens; metric tokens/s (whole node).
* ``--model resnet18`` ResNet-18, bf16 channels-last, synthetic 3x224x224 images, DDP, SGD+momentum;
                       metric images/s (whole node).

Invoked through ``python bench.py --model {gpt2,resnet18} ...``.
"""
from __future__ import annotations

import json
import os
import sys
import time


_NUMA = [None]   # the PCI address whose NUMA node this process is pinned to (bench.py), once verified


def _setup(shared_gpu: bool = False, numa_bdf=None):
    """(torch, dist, rank, world, device).  ``shared_gpu``: the one-GPU rehearsal of the N > 1 path --
    every rank on cuda:0, a gloo control group, DDP's bucket all-reduces and buffer broadcasts on the
    xGMI peer kernel (in place over the registered flat gradients)."""
    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pytorch_distributed_example_amd import dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = 0 if shared_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    from pytorch_distributed_example_amd.utils.stdio import stdout_to_stderr

    torch.cuda.set_device(local_rank)
    if numa_bdf:
        from pytorch_distributed_example_amd.utils.hipsched import verify_numa_binding
        _NUMA[0] = numa_bdf if verify_numa_binding(numa_bdf, local_rank) else None
    if world > 1 and not dist.is_initialized():
        with stdout_to_stderr():                  # RCCL's init banner must not precede the JSON line
            dist.init_process_group("gloo" if shared_gpu else "nccl", init_method="env://", rank=rank,
                                    world_size=world)
            dist.barrier()
    return torch, dist, rank, world, torch.device("cuda", local_rank)


def _w1_comm_group(dist):
    """A one-rank RCCL process group for the W = 1 rehearsal of the DDP communication path."""
    if not dist.is_initialized():
        from pytorch_distributed_example_amd.utils.stdio import stdout_to_stderr
        with stdout_to_stderr():    # port 0: the store binds an ephemeral port itself (no probe race)
            dist.init_process_group("nccl", init_method="tcp://127.0.0.1:0", rank=0, world_size=1)


def _comm_figure_wanted(args, world) -> bool:
    cf = getattr(args, "comm_figure", "auto")
    return world == 1 and not getattr(args, "force_comm", False) and cf in ("auto", "on")


def _graph_wanted(args) -> bool:
    """Whole-step hipGraph: on by default at every world size (DDP's collectives are captured as graph
    nodes, parallel/ddp.py); --model-graph off keeps eager launches."""
    return getattr(args, "model_graph", "auto") in ("auto", "on")


def _cap(args) -> float:
    """Initial DDP bucket cap (MB); 'auto' starts at 25 MB and ``tune_buckets`` sweeps at W>1."""
    return 25.0 if str(args.bucket_mb) == "auto" else float(args.bucket_mb)


def _tune(ddp, step, world, args, restore=None) -> dict:
    """W > 1 with --bucket-mb auto: time whole steps per (reduction route, bucket cap) (max over ranks),
    keep the fastest; the trial steps' training state is restored.  Reports the chosen cap and route,
    the per-candidate timings and the gradient bytes each rank hands to the all-reduce per step."""
    if not getattr(ddp, "comm_on", False):
        return {"bucket_mb": None, "grad_allreduce": "none"}
    from pytorch_distributed_example_amd.parallel import tune_bucket_cap
    out = {}
    if str(args.bucket_mb) == "auto":
        # shared-GPU rehearsal: only the peer route is device-side (gloo host collectives cannot be
        # captured into the step graph)
        routes = ["peer"] if getattr(args, "shared_gpu", False) else None
        timings, best = tune_bucket_cap(ddp, step, routes=routes, restore=restore)
        out.update(bucket_mb=best, bucket_sweep_ms_per_step=timings)
    else:
        out["bucket_mb"] = float(args.bucket_mb)
    out["grad_reduce_route"] = ddp.reduce_route
    out["peer_inplace"] = bool(getattr(ddp, "peer_inplace", False))
    out["grad_reduce_dtype"] = str(ddp.reduce_dtype or "param dtype").replace("torch.", "")
    out["grad_allreduce_bytes_per_step"] = ddp.wire_bytes_per_step()
    out["n_buckets"] = len(ddp.buckets)
    if ddp.peer_reason:
        out["peer_reason"] = ddp.peer_reason
    return out


def _timed(torch, dist, world, step, warmup, steps):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def _capture_step(torch, eager_step, sx, sy, ddp=None):
    """Capture ``eager_step(sx, sy)`` (forward, loss, backward with the DDP bucket collectives,
    optimizer) into one hipGraph after two allocator / autograd warm-up steps on a side stream."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            eager_step(sx, sy)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static_loss = eager_step(sx, sy)
    return graph, static_loss


def _gpt2_run(args, torch, dist, rank, world, dev, comm):
    """One timed GPT-2 run (``comm``: DDP wrapper with the full communication path, also at W = 1)."""
    from pytorch_distributed_example_amd.models import GPTConfig, build_gpt2
    from pytorch_distributed_example_amd.optim import AdamWMaster
    from pytorch_distributed_example_amd.parallel import DistributedDataParallel

    B = args.batch_size if args.batch_size != 128 else 16      # per-GPU micro-batch (sequences)
    T = args.seq_len
    cfg = GPTConfig(block_size=max(1024, T))
    model = build_gpt2(cfg, seed=args.seed, device=dev)
    ddp = DistributedDataParallel(model, bucket_cap_mb=_cap(args), force_comm=world == 1) if comm else model
    use_graph = _graph_wanted(args)
    opt = AdamWMaster(model.decay_groups(0.1), lr=6e-4, betas=(0.9, 0.95), max_grad_norm=1.0,
                      capturable=use_graph)
    # a pool of 256 sequences per rank of a learnable synthetic language, sharded by the framework's
    # DistributedSampler and reshuffled every epoch (set_epoch): no fixed handful of batches to
    # memorise.  The whole pool and the per-epoch shard orders of every epoch the run can reach are
    # built before timing, so a step only gathers its B rows on the device (no host sync, no randperm
    # inside the timed region).
    from pytorch_distributed_example_amd.data import DistributedSampler, synthetic_tokens
    pool = 256 * world
    data = synthetic_tokens(torch.arange(pool), T, cfg.vocab_size, seed=args.seed, device=dev)   # [pool, T+1]
    sampler = DistributedSampler(range(pool), num_replicas=world, rank=rank, shuffle=True, seed=args.seed)
    nb = sampler.num_samples // B
    n_epochs = (args.warmup + args.steps + 64 * (world > 1)) // nb + 2
    orders = []
    for e in range(n_epochs):
        sampler.set_epoch(e)
        orders.append(sampler.indices_tensor().long())
    orders = torch.stack(orders).to(dev)                 # [epochs, pool / world]
    it = [0]
    losses = []
    from pytorch_distributed_example_amd._ext import kernels
    K = kernels()
    sx = torch.empty(B, T, device=dev, dtype=torch.long)          # static model inputs / targets
    sy = torch.empty(B, T, device=dev, dtype=torch.long)
    ones = torch.ones((), device=dev, dtype=torch.float32)        # d loss / d loss (no fill kernel per step)

    def eager_step(x, y):
        opt.zero_grad()
        loss = ddp(x, y)
        loss.backward(ones)
        opt.step()
        return loss.detach()

    def next_batch():
        """The step's B sequences, gathered on the device by the framework's kernel into the static
        [B, T] inputs / targets (no index_select, no strided copies)."""
        e, j = divmod(it[0], nb)
        it[0] += 1
        K.token_batch(data, orders[e % n_epochs, j * B:(j + 1) * B], sx, sy)

    def step():
        next_batch()
        losses.append(eager_step(sx, sy))

    step0 = opt._step
    extra = _tune(ddp, step, world, args, restore=list(model.parameters()) + opt.state_tensors()) if comm else \
        {"bucket_mb": None, "grad_allreduce": "none"}
    opt._step = step0
    if getattr(opt, "capturable", False):
        opt.state_tensors()[-1].fill_(float(step0))
    if use_graph:
        # the whole step (forward, loss, backward with the DDP bucket all-reduces, grad-norm clip, AdamW
        # with its device-side step count) is captured once into a hipGraph and replayed: ~340 launches
        # per step leave the host and the inter-kernel gaps shrink.  Each step gathers its batch into
        # the static input first (inside the timed region).
        next_batch()
        graph, static_loss = _capture_step(torch, eager_step, sx, sy)

        def step():                                  # noqa: F811 - the graph-replay step
            next_batch()
            graph.replay()
            losses.append(static_loss)

        graph.replay()                               # first launch of the graph outside the timed window
        extra["mode"] = "hipgraph (whole step" + (", DDP collectives captured)" if comm else ")")
    else:
        extra["mode"] = "eager"
    elapsed = _timed(torch, dist, world, step, args.warmup, args.steps)
    if comm:
        ddp.check_health()
    return {"elapsed": elapsed, "extra": extra, "B": B, "T": T, "flops_per_token": model.flops_per_token(),
            "last_loss": float(losses[-1])}


def bench_gpt2(args):
    torch, dist, rank, world, dev = _setup(getattr(args, "shared_gpu", False), getattr(args, "numa_bdf", None))
    r = _gpt2_run(args, torch, dist, rank, world, dev, comm=world > 1 or getattr(args, "force_comm", False))
    B, T = r["B"], r["T"]
    tps = args.steps * B * T * world / r["elapsed"]
    out = {
        "metric": "tokens/sec (whole node), GPT-2-small DDP",
        "value": round(tps, 1), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic learnable token sequences (next = 31*prev+7+U[0,4) mod V; loss floor ln 4), "
                "256 per rank sharded by DistributedSampler, reshuffled per epoch, random-init weights",
        "config": {"model": "GPT-2 small 124M (12L, 12H, d768, ctx 1024, vocab 50257->50304)",
                   "global_batch": B * world, "per_gpu_batch": B, "seq_len": T, "parallelism": f"dp{world}",
                   "host_cpus": f"NUMA node of GPU {_NUMA[0]}" if _NUMA[0] else "unpinned",
                   "optimizer": "AdamW(fp32 master, wd 0.1, clip 1.0)", **r["extra"]},
        "model_tflops_per_gpu": round(r["flops_per_token"] * tps / world / 1e12, 1),
        "last_loss": round(r["last_loss"], 4),
    }
    if _comm_figure_wanted(args, world):
        # the same step with an RCCL communicator and DDP's whole communication path (bucket all-reduces
        # captured into the step graph) at W = 1: what the W > 1 path costs besides the wire time
        try:
            _w1_comm_group(dist)
            r2 = _gpt2_run(args, torch, dist, rank, world, dev, comm=True)
            out["w1_rccl_comm"] = {"value": round(args.steps * B * T / r2["elapsed"], 1),
                                   "ms_per_step": round(r2["elapsed"] / args.steps * 1e3, 3), **r2["extra"]}
        except Exception as e:   # noqa: BLE001 - the headline stands; report the secondary failure
            out["w1_rccl_comm"] = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0:
        from pytorch_distributed_example_amd.utils.stdio import emit_result
        emit_result(out)
    if dist.is_initialized():
        dist.destroy_process_group()


def run_model_bench(args):
    if args.model == "gpt2":
        return bench_gpt2(args)
    if args.model == "resnet18":
        from bench_resnet import bench_resnet18
        return bench_resnet18(args)
    raise ValueError(args.model)
