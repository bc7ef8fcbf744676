#!/usr/bin/env python3
"""Headline benchmark: whole-node training throughput of the reference toy CNN on MI355X.

Metric (BASELINE.json): images/sec for the whole node, toy CNN (``Net``, /root/reference/mnist/
main.py:130-147) on synthetic MNIST, DDP at 1/2/4/8 GPUs (weak scaling: 128 images per GPU per
step, the reference's default ``--batch-size``), fp32 (the reference's dtype), Adam(lr=1e-3).

One timed "step" is the full reference step (main.py:84-99): forward, cross-entropy, backward,
gradient all-reduce + average over ranks (bucketed, overlapped with the conv backward; each bucket
takes the faster of RCCL and the xGMI peer all-reduce, timed on this node at start-up),
Adam update, loss/accuracy meters.  Each rank trains on its DistributedSampler shard of a
60,000-sample synthetic set (random-init weights, synthetic data: no network on the box).

  python bench.py --gpus N --steps K --warmup W
  (N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N ...,
   or the same command without a launcher: bench.py then starts the N ranks itself and relays rank 0's
   line; a launch whose WORLD_SIZE differs from --gpus is refused with an error line, exit code 2)

Every captured hipGraph -- at both step parities of the prefetching engine, so no warm-up / step count
can leave a capture or first launch for the timed window -- is replayed (``--prime-replays``, default
3) before the W untimed warm-up steps; then exactly K steps are timed,
bracketed by barrier + device synchronize on both sides; the elapsed time is the MAX over ranks;
rank 0 prints one JSON line.  A failure still prints one JSON line (``value`` null, ``error``) and
exits non-zero, and so does a communication-health failure (peer barrier time-out, RCCL error):
a poisoned peer path skips its barriers and would otherwise report an inflated number.

At N>1 every rank first times the comm-free single-GPU step on its own GPU (all ranks at once,
before the communicator exists): the same-job W=1 anchor.  The line then carries
``w1_anchor_images_per_s`` (mean over ranks), ``scaling_eff_same_job`` = (value / N) / anchor, and
``per_rank``: every rank's device (index, UUID), RCCL communicator size and device, and peer-path
status, all-gathered; a repeated device or an RCCL communicator whose size is not N (the reference's
every-rank-on-GPU-0 bug, /root/reference/mnist/main.py:181-182) fails the run with an error line.

At W=1 the line also carries ``w1_rccl_comm``: the same step measured a second time with an RCCL
communicator initialised and the full W>1 communication path running (config 2 of BASELINE.json:
"DDP world_size=1 ... RCCL init + HIP kernels"); the headline ``value`` stays the comm-free step.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import socket
import sys
import time
import traceback

BASELINE_METRIC = "images/sec (whole node) + DDP scaling eff, toy CNN synthetic MNIST 1/2/4/8 GPU"
STOCK_TORCH_W1 = 121442.1   # same-hardware stock-PyTorch reference loop, W=1 (profiles/baseline/)


def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch-size", type=int, default=128, help="per-GPU batch (reference default 128)")
    ap.add_argument("--mode", choices=["graph", "eager"], default="graph")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="steps captured per hipGraph (graph mode); 0 = the largest divisor of --steps <= 100")
    ap.add_argument("--no-overlap", action="store_true", help="one all-reduce after backward (no bucketing)")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="rehearsal only: every rank on cuda:0, gloo control group, peer all-reduce for the data")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the W>1 communication path (buckets, routes, split optimizer) even at W=1")
    ap.add_argument("--no-autotune", action="store_true", help="W>1: skip the whole-step schedule autotuning")
    ap.add_argument("--schedule", default=None,
                    help="force one communication schedule by its autotuner label, e.g. 'serial 431296:peer1' "
                         "(no autotuning; traces and A/B runs)")
    ap.add_argument("--autotune-budget-s", type=float, default=60.0,
                    help="wall-clock budget of the schedule autotuner (candidates left untimed past it)")
    ap.add_argument("--prime-replays", type=int, default=3,
                    help="untimed replays of each captured graph before the warm-up steps")
    ap.add_argument("--clock-warm-ms", type=float, default=0.0,
                    help="untimed back-to-back training steps (about this many ms of GPU work) right before the "
                         "W warm-up steps, so the timed window starts at the clock a sustained run holds "
                         "(0 = off; PDE_BENCH_CLOCK_WARM_MS overrides)")
    ap.add_argument("--lead-steps", type=int, default=int(os.environ.get("PDE_BENCH_LEAD", "1")),
                    help="graph mode: the first L timed steps replay as 1-step graphs ahead of the multi-step "
                         "graphs, so the GPU starts while the host still submits the long graph (0 = off)")
    ap.add_argument("--comm-figure", choices=["auto", "on", "off"], default="auto",
                    help="W=1: also time the step with RCCL initialised + the comm path on (auto = on at W=1)")
    ap.add_argument("--train-size", type=int, default=60000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--model", choices=["lenet", "gpt2", "resnet18"], default="lenet",
                    help="lenet = the BASELINE headline (default); gpt2 / resnet18 = the driver-added configs")
    ap.add_argument("--no-spin-wait", action="store_true",
                    help="leave HIP's default host wait policy (default: hipDeviceScheduleSpin, utils/hipsched.py)")
    ap.add_argument("--seq-len", type=int, default=1024, help="gpt2: sequence length")
    ap.add_argument("--model-graph", choices=["auto", "on", "off"], default="auto",
                    help="gpt2 / resnet18: replay the whole training step (fwd + bwd + optimizer, with DDP's "
                         "bucket all-reduces and buffer broadcast captured as graph nodes at W>1) as one "
                         "hipGraph; auto = on at every world size, off = eager launches")
    ap.add_argument("--bucket-mb", type=str, default="auto",
                    help="gpt2/resnet18: DDP gradient bucket cap in MB, or 'auto' (timed sweep at W>1)")
    return ap


def _graph_steps(args, n=None) -> int:
    """Steps per captured hipGraph for a run of n steps (default --steps): fewer, longer graphs mean
    fewer graph-to-graph transitions (~13 us each, profiles/r3_window/) -- --steps 20 is one replay
    of a 20-step graph, --warmup 5 one replay of a 5-step graph."""
    if args.graph_steps > 0 and n is None:
        return args.graph_steps
    n = args.steps if n is None else n
    return max(d for d in range(1, min(100, max(1, n)) + 1) if n % d == 0)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _replay_plan(n: int, S: int, lead: int = 0) -> list:
    """Graph lengths replayed for n steps: ``lead`` 1-step graphs, then S-step graphs, then one graph of
    the remainder."""
    full, r = divmod(n - lead, S)
    return [1] * lead + [S] * full + ([r] if r else [])


def _graph_plan(args, S: int) -> str:
    """The timed window's replays as reported in config.mode, e.g. 'graph replays of 1 + 19 steps'
    (--steps 20, one lead step) or 'graph replays of 1 + 100 x19 + 99 steps' (--steps 2000)."""
    L = min(max(args.lead_steps, 0), args.steps)
    full, r = divmod(args.steps - L, S)
    parts = ["1"] * L + ([str(S) if full == 1 else f"{S} x{full}"] if full else []) + ([str(r)] if r else [])
    return f"graph replays of {' + '.join(parts)} steps"


class _Job:
    """Per-process state shared by the headline run and the W=1 comm figure."""

    def __init__(self, args):
        self.args = args
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_rank = 0 if args.shared_gpu else int(os.environ.get("LOCAL_RANK", "0"))
        self.spin_wait = False
        self.numa = None


def _comm_info(dist, comm, eng):
    """What the communication path actually ran on (proof that RCCL saw N ranks)."""
    if comm is None:
        return {}
    info = {"rccl_world": None, "rccl_device": None, "peer_ok": comm.peer is not None,
            "peer_inplace": bool(getattr(comm, "peer_inplace", False))}
    rc = comm.group.rccl
    if rc is not None:
        try:
            info["rccl_world"] = rc.comm_count()
            info["rccl_device"] = rc.cu_device()
        except Exception as e:   # noqa: BLE001 - report, never fail the bench on a query
            info["rccl_query_error"] = str(e)
    if comm.peer is None:
        reason = getattr(comm, "peer_reason", "")
        if reason:
            info["peer_reason"] = reason
    if eng is not None and eng.comm_on:
        info["schedule"] = getattr(eng, "schedule", eng.mode)
        info["routes"] = {str(k): v for k, v in comm.routes.items()}
        info["route_us_per_call"] = {str(k): v for k, v in comm.timings.items()}
    return info


def _device_id(local_rank: int) -> str:
    """A node-unique identity of this rank's GPU (UUID, else PCI bus id, else the index)."""
    if os.environ.get("PDE_BENCH_STUB") == "1":        # CPU control-flow rehearsal (tests)
        return os.environ.get("PDE_BENCH_STUB_DEV", f"stub-gpu-{local_rank}")
    import torch

    props = torch.cuda.get_device_properties(local_rank)
    for attr in ("uuid", "pci_bus_id"):
        v = getattr(props, attr, None)
        if v not in (None, "", 0):
            return f"{attr}:{v}"
    return f"index:{local_rank}"


def _rank_row(job: _Job, comm) -> dict:
    info = _comm_info(None, comm, None) if comm is not None else {}
    return {"rank": job.rank, "local_rank": job.local_rank, "host": socket.gethostname(),
            "device": job.local_rank, "device_id": _device_id(job.local_rank),
            "rccl_world": info.get("rccl_world"), "rccl_device": info.get("rccl_device"),
            "peer_ok": info.get("peer_ok"), "peer_reason": info.get("peer_reason", "")[:200]}


def _gather_rows(row: dict, world: int) -> list:
    """All-gather one JSON-able dict per rank over the host control path (fixed-size byte image)."""
    import torch

    from pytorch_distributed_example_amd import dist

    if world == 1 or not dist.is_initialized():
        return [row]
    width = 1024
    b = json.dumps(row).encode()[:width]
    t = torch.zeros(world, width, dtype=torch.int32)        # one row per rank, summed = concatenated
    t[job_rank(row)][: len(b)] = torch.tensor(list(b), dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [json.loads(bytes(r[r > 0].tolist()).decode()) for r in t]


def job_rank(row: dict) -> int:
    return int(row["rank"])


def validate_ranks(rows: list, world: int, shared_gpu: bool = False) -> str:
    """'' if every rank ran on its own GPU with an N-rank communicator, else what is wrong
    (``shared_gpu``: the one-GPU rehearsal, where every rank is on cuda:0 by design)."""
    if len(rows) != world or sorted(r["rank"] for r in rows) != list(range(world)):
        return f"expected {world} rank rows, got ranks {sorted(r.get('rank') for r in rows)}"
    seen = {}
    for r in rows if not shared_gpu else []:
        key = (r["host"], r["device_id"])
        if key in seen:
            return (f"ranks {seen[key]} and {r['rank']} share one GPU ({r['device_id']} on {r['host']}): "
                    f"every rank must own a device")
        seen[key] = r["rank"]
    for r in rows:
        if r.get("rccl_world") is not None and r["rccl_world"] != world:
            return f"rank {r['rank']}: RCCL communicator has {r['rccl_world']} ranks, not {world}"
        if r.get("rccl_device") is not None and r["rccl_device"] != r["device"]:
            return f"rank {r['rank']}: RCCL communicator on device {r['rccl_device']}, rank on {r['device']}"
    ok = {bool(r.get("peer_ok")) for r in rows}
    if len(ok) > 1:
        return "the xGMI peer path is enabled on some ranks only (the set-up vote must be collective)"
    return ""


class _StubEngine:
    """PDE_BENCH_STUB=1 (CPU tests only): the engine surface ``bench.py`` drives, with a sleep per
    step instead of GPU kernels, so the N>1 control flow (self-launch, anchor, gather, validation,
    the JSON line) runs on a machine without a GPU.  Its numbers are not measurements."""

    def __init__(self, comm):
        self.comm, self.comm_on, self.mode, self.samples = comm, comm is not None, "stub", 0

    def replay(self, B=None, steps=1):
        time.sleep(50e-6 * steps)
        if self.comm is not None:
            import torch

            from pytorch_distributed_example_amd import dist
            dist.all_reduce(torch.zeros(1))

    def step(self, B=None):
        self.replay(B, 1)

    def prime_graphs(self, *a, **k):
        pass

    def reset_meters(self):
        pass

    def read_meters(self, reset=True):
        return 0.0, 0, 0


def _init_group(job: _Job):
    """The job's process group (RCCL; gloo for the shared-GPU rehearsal and the CPU stub)."""
    from pytorch_distributed_example_amd import dist
    from pytorch_distributed_example_amd.utils.stdio import stdout_to_stderr

    if dist.is_initialized():
        return
    if "MASTER_PORT" in os.environ:
        init = "env://"
    else:   # W = 1: port 0 lets the store bind an ephemeral port (a probed port can be taken meanwhile)
        init = f"tcp://127.0.0.1:{0 if job.world == 1 else _free_port()}"
    backend = "gloo" if job.args.shared_gpu or os.environ.get("PDE_BENCH_STUB") == "1" else "nccl"
    with stdout_to_stderr():                      # RCCL's init banner must not precede the JSON line
        dist.init_process_group(backend, init_method=init, rank=job.rank, world_size=job.world)


def _run_lenet(job: _Job, force_comm: bool, steps: int, warmup: int, comm_world: bool, max_over_ranks: bool = True):
    """Builds the engine, times ``steps`` steps, returns (elapsed_s, eng, comm, extra)."""
    import torch

    from pytorch_distributed_example_amd import dist
    from pytorch_distributed_example_amd.data import DistributedSampler, synthetic_mnist
    from pytorch_distributed_example_amd.engine import LeNetTrainStep
    from pytorch_distributed_example_amd.models import build_net
    from pytorch_distributed_example_amd.utils.stdio import stdout_to_stderr

    args, world, rank = job.args, job.world, job.rank
    comm = None
    if os.environ.get("PDE_BENCH_STUB") == "1":
        if comm_world:
            _init_group(job)
        eng = _StubEngine(True if comm_world and world > 1 else None)
        return _timed_window(job, eng, None, {}, lambda n, S=1, lead=0: eng.replay(steps=n), steps, warmup,
                             max_over_ranks=max_over_ranks)
    dev = torch.device("cuda", job.local_rank)
    with stdout_to_stderr():                      # RCCL's init banner must not precede the JSON line
        if comm_world:
            _init_group(job)
            comm = dist.engine_comm(allow_host_only=args.shared_gpu)
        net = build_net(seed=args.seed, device=dev)
        if comm is not None:
            dist.broadcast_parameters(net)            # DDP semantics: replicas start identical
        eng = LeNetTrainStep(net, batch_size=args.batch_size, lr=1e-3, comm=comm, overlap=not args.no_overlap,
                             force_comm=force_comm)
    train = synthetic_mnist(args.train_size, seed=args.seed, device=dev, kind="fashion")
    eng.bind_dataset(train.images, train.labels)
    sampler = DistributedSampler(train, num_replicas=world, rank=rank, shuffle=True, seed=args.seed)
    idx = sampler.indices_tensor()
    nfull = idx.numel() // args.batch_size
    eng.set_epoch_indices(idx[: nfull * args.batch_size])   # full batches only: every timed step is B=128

    S = _graph_steps(args)
    Sw = _graph_steps(args, args.warmup) if args.warmup > 0 else 1
    extra = {}

    # timed window: L lead steps (1-step graphs: a short graph starts on the GPU ~10 us sooner than a
    # 20-step one, and the long graph's submission then overlaps the lead step), then graphs of S steps
    # and one graph of the remainder (profiles/r6_lenet/lead_step/)
    L = min(max(args.lead_steps, 0), steps) if args.mode == "graph" else 0
    r_timed = (steps - L) % S

    def run(n, S=S, lead=0):
        if args.mode == "graph":
            for k in _replay_plan(n, S, lead):
                eng.replay(steps=k)             # every length in the plan is primed below
        else:
            for _ in range(n):
                eng.step()

    if eng.comm_on and args.schedule:
        eng.set_schedule(args.schedule)
    elif eng.comm_on and not args.no_autotune:
        # time every communication schedule (bucket routes x overlap) on whole steps, keep the fastest
        extra["schedule_us_per_step"] = eng.autotune_schedule(graph_steps=S, budget_s=args.autotune_budget_s)
        extra["compute_only_us_per_step"] = eng.compute_only_us   # same step, collectives left out
        health = comm.health()
        if health:
            raise RuntimeError(f"communication failure during schedule autotuning: {health}")
    gc_off = os.environ.get("PDE_BENCH_GC") != "1"
    if gc_off:       # as timeit does: no Python GC pause between graph launches inside the window;
        gc.collect()     # collected BEFORE the priming / warm-up, so the GPU does not idle (and clock
        gc.disable()     # down) for the collection between the last warm-up step and the timed window
    if args.mode == "graph":
        # both step parities of both graphs are captured and launched once before the warm-up, so no
        # warm-up / step count can make the timed window capture or first-launch a graph
        eng.prime_graphs(tuple(sorted({S, Sw, r_timed or 1, 1})), replays=max(1, args.prime_replays))
    _clock_warm(args, eng, run, S)
    try:
        return _timed_window(job, eng, comm, extra, run, steps, warmup, Sw, max_over_ranks=max_over_ranks, lead=L)
    finally:
        if gc_off:
            gc.enable()


def _clock_warm(args, eng, run, S):
    """Optional untimed back-to-back training steps (``--clock-warm-ms`` of GPU work, enqueued without
    a host sync) right before the W warm-up steps, to start the timed window at a sustained-load clock.
    Off by default: measured on MI355X it did not move the 20-step window (57.3 / 57.5 us/step with
    20 ms of warm steps vs 56.8 / 57.9 without, same box, profiles/r4_lenet/)."""
    warm_ms = float(os.environ.get("PDE_BENCH_CLOCK_WARM_MS", args.clock_warm_ms))
    if warm_ms <= 0:
        return
    n = max(1, int(round(warm_ms * 1e3 / 55.0)))        # ~55 us per toy-CNN step on one MI355X
    n = ((n + S - 1) // S) * S
    run(n, S)


_BARRIER_T = {}


def _device_barrier(comm, dist):
    """Barrier for the window brackets: an RCCL all-reduce of one element + synchronize when the group
    has RCCL (every rank must arrive; the GPU idles for microseconds, not for a host TCP round trip
    that lets the clocks drop before the timed window), else the host barrier."""
    import torch

    if dist.get_world_size() == 1:          # a barrier over one rank is the device synchronize alone
        torch.cuda.synchronize()
        return
    rc = comm.group.rccl if comm is not None else None
    if rc is None:
        dist.barrier()
        return
    t = _BARRIER_T.get(rc.device)
    if t is None:
        t = _BARRIER_T[rc.device] = torch.zeros(1, device=torch.device("cuda", rc.device))
    dist.all_reduce(t)
    torch.cuda.synchronize()


def _timed_window(job, eng, comm, extra, run, steps, warmup, Sw=1, max_over_ranks=True, lead=0):
    """W warm-up steps, then exactly K timed steps bracketed by barrier + device synchronize on both
    sides.  ``max_over_ranks``: the elapsed time is the MAX over ranks (the job's step time); off for
    the per-rank W=1 anchor, whose ranks still start together (host barrier) but time alone."""
    import torch

    from pytorch_distributed_example_amd import dist

    stub = os.environ.get("PDE_BENCH_STUB") == "1"
    sync = (lambda: None) if stub else torch.cuda.synchronize
    world = job.world
    grouped = dist.is_initialized() and world > 1
    run(warmup, Sw)
    # meters cover the timed steps only: zeroed on the stream (no .item() round trips: every idle
    # microsecond before the window lets the GPU clock down, profiles/r3_window/)
    eng.reset_meters()
    sync()
    if comm is not None:
        _device_barrier(comm, dist)
    elif grouped:
        dist.barrier()
    sync()
    trace = os.environ.get("PDE_BENCH_TRACE") == "1" and not stub
    if trace:       # diagnostics only: GPU-clocked window and host launch time, to stderr
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    t0 = time.perf_counter()
    run(steps, lead=lead)
    t_launch = time.perf_counter() - t0
    if trace:
        ev1.record()
    sync()
    t_end = time.perf_counter()
    if comm is not None:
        _device_barrier(comm, dist)
        sync()
        t_end = time.perf_counter()
    elif grouped and max_over_ranks:
        dist.barrier()
    elapsed = (time.perf_counter() if max_over_ranks else t_end) - t0
    if trace:
        print(json.dumps({"trace_host_us": round(elapsed * 1e6, 1), "trace_launch_us": round(t_launch * 1e6, 1),
                          "trace_gpu_us": round(ev0.elapsed_time(ev1) * 1e3, 1)}), file=sys.stderr)
    if grouped and max_over_ranks:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if comm is not None:
        health = comm.health()
        if health:
            raise RuntimeError(f"communication failure during the timed steps: {health}")
    return elapsed, eng, comm, extra


def _w1_anchor(job: _Job):
    """N>1: every rank times the comm-free single-GPU step on its own GPU, all at once (host barrier
    before the window), before the communicator exists.  Returns the per-rank images/s list."""
    import torch

    from pytorch_distributed_example_amd import dist

    args = job.args
    e, eng, _, _ = _run_lenet(job, False, args.steps, args.warmup, comm_world=False, max_over_ranks=False)
    v = torch.zeros(job.world, dtype=torch.float64)
    v[job.rank] = args.steps * args.batch_size / e
    dist.all_reduce(v, op=dist.ReduceOp.SUM)
    del eng
    gc.collect()
    if os.environ.get("PDE_BENCH_STUB") != "1":
        torch.cuda.synchronize()
    return [round(x, 1) for x in v.tolist()]


def lenet_main(job: _Job):
    import torch

    from pytorch_distributed_example_amd import dist

    args, world, rank = job.args, job.world, job.rank
    stub = os.environ.get("PDE_BENCH_STUB") == "1"
    if not stub:
        torch.cuda.set_device(job.local_rank)
        if job.numa:
            from pytorch_distributed_example_amd.utils.hipsched import verify_numa_binding
            if not verify_numa_binding(job.numa, job.local_rank):
                job.numa = None           # KFD order is not the runtime's device order: unpinned
    comm_world = world > 1 or args.force_comm
    anchors = None
    if world > 1:
        _init_group(job)                  # the group first: the anchor's ranks start together
        anchors = _w1_anchor(job)
    elapsed, eng, comm, extra = _run_lenet(job, args.force_comm, args.steps, args.warmup, comm_world)
    rows = _gather_rows(_rank_row(job, comm), world)
    bad = validate_ranks(rows, world, args.shared_gpu) if world > 1 else ""
    if bad:
        raise RuntimeError(f"rank placement check failed: {bad}")
    loss_sum, correct, _ = eng.read_meters()
    n_img = args.steps * args.batch_size * world
    ips = n_img / elapsed
    S = _graph_steps(args)
    out = {
        "metric": BASELINE_METRIC,
        "value": round(ips, 1),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (class-conditional MNIST-shaped, device resident), random-init weights",
        "config": {
            "model": "toy CNN Net (conv5x5 20 -> conv5x5 50 -> fc 500 -> fc 10), 431,080 params",
            "global_batch": args.batch_size * world,
            "per_gpu_batch": args.batch_size,
            "seq_len": None,
            "parallelism": f"dp{world}",
            "optimizer": "Adam(lr=1e-3)",
            "mode": args.mode if args.mode == "eager" else _graph_plan(args, S),
            "grad_allreduce": "none" if not eng.comm_on else eng.mode,
            "host_wait": "spin" if job.spin_wait else "runtime default",
            "host_cpus": f"NUMA node of GPU {job.numa}" if job.numa else "unpinned",
            **_comm_info(dist, comm, eng),
            **extra,
        },
        "stock_torch_same_hw_w1_images_per_s": STOCK_TORCH_W1,
        "speedup_vs_stock_torch_per_gpu": round(ips / world / STOCK_TORCH_W1, 2),
        "train_loss_mean_timed_rank0": round(loss_sum / max(1, args.steps * args.batch_size), 5),
        "train_acc_timed_rank0": round(correct / max(1, args.steps * args.batch_size), 5),
        "per_rank": rows,
    }
    if anchors:
        a1 = sum(anchors) / len(anchors)
        out["w1_anchor_images_per_s"] = round(a1, 1)
        out["w1_anchor_per_rank"] = anchors
        out["scaling_eff_same_job"] = round(ips / world / a1, 4)
    if stub:
        out["data"] = "STUB (PDE_BENCH_STUB=1: CPU control-flow test, sleep per step, not a measurement)"
    want_fig = args.comm_figure == "on" or (args.comm_figure == "auto" and world == 1 and not args.force_comm)
    if want_fig and world == 1:
        # config 2 (BASELINE.json): the same step with RCCL initialised and the comm path running
        try:
            e2, eng2, comm2, extra2 = _run_lenet(job, True, args.steps, args.warmup, True)
            out["w1_rccl_comm"] = {"value": round(args.steps * args.batch_size / e2, 1),
                                   "ms_per_step": round(e2 / args.steps * 1e3, 5),
                                   "grad_allreduce": eng2.mode, **_comm_info(dist, comm2, eng2), **extra2}
        except Exception as e:   # noqa: BLE001 - the headline stands; report the secondary failure
            out["w1_rccl_comm"] = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0:
        from pytorch_distributed_example_amd.utils.stdio import emit_result
        emit_result(out)
    if dist.is_initialized():
        dist.destroy_process_group()


def _error_line(args, world, msg: str) -> dict:
    return {"metric": BASELINE_METRIC if args.model == "lenet" else args.model, "value": None,
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "error": msg}


def _self_launch(args, argv) -> int:
    """``--gpus N`` (N > 1) without a launcher: start N rank processes of this script, one per GPU
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1, env:// rendezvous, the launcher's
    gang-kill on the first failure), and relay rank 0's JSON line on this process's stdout.  The
    parent makes no HIP call (it never imports torch); the ranks' own stdout goes to stderr so the
    relayed line stays the only one here."""
    import tempfile

    from pytorch_distributed_example_amd.launch import free_port, run_gang

    fd, result = tempfile.mkstemp(prefix="pde_bench_", suffix=".json")
    os.close(fd)
    try:
        cmd = [sys.executable, os.path.abspath(__file__)] + list(argv)
        rc = run_gang(cmd, args.gpus, "127.0.0.1", free_port(), extra_env={"PDE_BENCH_RESULT": result},
                      stdout=sys.stderr)
        with open(result) as f:
            line = f.read().strip()
    finally:
        os.unlink(result)
    if line:
        print(line, flush=True)
    else:
        print(json.dumps(_error_line(args, args.gpus, f"rank 0 reported no result (gang exit code {rc})")),
              flush=True)
    return rc if rc else (0 if line else 1)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = build_parser().parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(_self_launch(args, argv))
    job = _Job(args)
    print(f"[bench] rank {job.rank}/{job.world} local_rank {job.local_rank} pid {os.getpid()}", file=sys.stderr,
          flush=True)
    if job.world != args.gpus:
        # a mislabelled run (e.g. --gpus 8 on a 1-rank launch) must not report as the other config
        if job.rank == 0:
            print(json.dumps(_error_line(args, job.world, f"--gpus {args.gpus} but WORLD_SIZE={job.world}")),
                  flush=True)
        sys.exit(2)
    if os.environ.get("PDE_BENCH_NUMA", "1") != "0":
        # before any HIP call: host threads on the GPU's own socket (launch doorbells, sync polling)
        from pytorch_distributed_example_amd.utils.hipsched import bind_local_numa
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
        job.numa = bind_local_numa(job.local_rank, [0] * lws if args.shared_gpu else list(range(lws)))
    if not args.no_spin_wait:
        # before any HIP context exists: spinning host waits keep the graph-launch path fast
        from pytorch_distributed_example_amd.utils.hipsched import set_schedule
        job.spin_wait = set_schedule(job.local_rank)
    try:
        if args.model != "lenet":
            from bench_models import run_model_bench
            args.numa_bdf = job.numa
            return run_model_bench(args)
        return lenet_main(job)
    except Exception as e:   # noqa: BLE001 - always one JSON line, then a non-zero exit
        traceback.print_exc(file=sys.stderr)
        if job.rank == 0:
            from pytorch_distributed_example_amd.utils.stdio import emit_result
            emit_result(_error_line(args, job.world, f"{type(e).__name__}: {e}"))
        sys.exit(1)


if __name__ == "__main__":
    main()
