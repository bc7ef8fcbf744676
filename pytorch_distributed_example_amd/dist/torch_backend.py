"""The framework's runtime as a ``torch.distributed`` backend: ``backend="pde"``.

The reference drives ``torch.distributed`` directly (``import torch.distributed as dist`` ...
``dist.init_process_group(backend=args.backend, ...)``, /root/reference/mnist/main.py:198-204,
/root/reference/toy/main.py:28-33).  Importing this module registers a c10d backend named ``pde``,
so such code runs its collectives on the framework's native runtime -- RCCL communicators over xGMI
for GPU tensors (one per GPU, ``csrc/runtime/rccl_comm.cpp``) and the C++ TCP host collectives
for CPU tensors (``hostcomm.cpp``) -- by changing nothing but the backend string:

    import torch.distributed as dist
    import pytorch_distributed_example_amd.dist.torch_backend   # registers "pde"
    dist.init_process_group("pde", init_method="tcp://127.0.0.1:23456", rank=r, world_size=w)
    dist.all_reduce(t)                                           # -> framework runtime

Rendezvous rides on torch's own store only to publish the address of the framework's C++ store
(one server per job, on global rank 0); every group, including each ``new_group`` (the reference's
toy creates one per step, toy/main.py:16), gets its own HostComm / RCCL communicator keyed by a
job-unique id.  Collectives complete in order on the caller's stream (GPU) or synchronously
(CPU), so the returned Work is already complete -- exactly the reference's blocking usage.
"""
from __future__ import annotations

import os
import socket

import torch
import torch.distributed as tdist
from torch._C._distributed_c10d import (
    AllgatherOptions, AllreduceCoalescedOptions, AllreduceOptions, AllToAllOptions, BarrierOptions, BroadcastOptions,
    GatherOptions, ReduceOptions, ReduceScatterOptions, ScatterOptions, _create_work_from_future,
)
from torch.futures import Future

from .._ext import runtime
from . import api

_SERVER = None          # this process's StoreServer (global rank 0 only)
_CLIENT = None          # connection to the job's framework store
_ADDR_KEY = "pde_store_addr"


def _done(result=None):
    fut = Future()
    fut.set_result(result)
    return _create_work_from_future(fut)


def _op(opts):
    op = getattr(opts, "reduceOp", None)
    name = str(getattr(op, "op", op)).split(".")[-1].upper()     # RedOpType.SUM -> SUM
    return api.ReduceOp[name]


def _connect(prefix_store, rank: int, timeout_ms: int):
    global _SERVER, _CLIENT
    if _CLIENT is not None:
        return _CLIENT
    R = runtime()
    if rank == 0 and not prefix_store.check([_ADDR_KEY]):
        _SERVER = R.StoreServer("0.0.0.0", 0)
        host = os.environ.get("MASTER_ADDR") or socket.gethostbyname(socket.gethostname())
        prefix_store.set(_ADDR_KEY, f"{host}:{_SERVER.port}")
    addr = prefix_store.get(_ADDR_KEY).decode()
    host, port = addr.rsplit(":", 1)
    _CLIENT = R.StoreClient(host, int(port), timeout_ms)
    return _CLIENT


class PDEProcessGroup(tdist.ProcessGroup):
    """c10d ProcessGroup whose collectives run on the framework runtime (see module docstring)."""

    def __init__(self, prefix_store, rank: int, world_size: int, timeout):
        super().__init__(rank, world_size)
        timeout_ms = int((timeout or api.DEFAULT_TIMEOUT).total_seconds() * 1000)
        store = _connect(prefix_store, rank, timeout_ms)
        # a job-unique key space for this group: drawn once by group rank 0, shared via torch's store
        if rank == 0:
            prefix_store.set("pde_gid", str(store.add("pde/torch_groups", 1)))
        gid = prefix_store.get("pde_gid").decode()
        prefix = f"pde/tg{gid}"
        rccl, dev = None, None
        backend = api.Backend("gloo")
        if torch.cuda.is_available():
            dev = torch.cuda.current_device()
            rccl = api._make_rccl(store, prefix, rank, world_size, dev)
            backend = api.Backend("nccl")
        self._pg = api.ProcessGroup(list(range(world_size)), rank, backend, prefix, store, timeout_ms, rccl, dev)

    def getBackendName(self):
        return "pde"

    # --- collectives (tensor lists: one tensor per rank-local device, as c10d passes them) ---------
    def allreduce(self, tensor_list, opts=AllreduceOptions()):
        for t in tensor_list:
            api.all_reduce(t, _op(opts), group=self._pg)
        return _done(tensor_list)

    def allreduce_coalesced(self, tensor_list, opts=AllreduceCoalescedOptions()):
        return self.allreduce(tensor_list, opts)

    def broadcast(self, tensor_list, opts=BroadcastOptions()):
        for t in tensor_list:
            api.broadcast(t, opts.rootRank, group=self._pg)
        return _done(tensor_list)

    def allgather(self, output_tensors, input_tensor, opts=AllgatherOptions()):
        for outs, inp in zip(output_tensors, input_tensor):
            api.all_gather(outs, inp, group=self._pg)
        return _done(output_tensors)

    def _allgather_base(self, output, input, opts=AllgatherOptions()):
        api.all_gather_into_tensor(output, input, group=self._pg)
        return _done(output)

    def reduce_scatter(self, output_tensors, input_tensors, opts=ReduceScatterOptions()):
        for out, ins in zip(output_tensors, input_tensors):
            api.reduce_scatter(out, ins, _op(opts), group=self._pg)
        return _done(output_tensors)

    def _reduce_scatter_base(self, output, input, opts=ReduceScatterOptions()):
        api.reduce_scatter_tensor(output, input, _op(opts), group=self._pg)
        return _done(output)

    def reduce(self, tensor_list, opts=ReduceOptions()):
        for t in tensor_list:
            api.reduce(t, opts.rootRank, _op(opts), group=self._pg)
        return _done(tensor_list)

    def gather(self, output_tensors, input_tensors, opts=GatherOptions()):
        outs = output_tensors[0] if output_tensors else None
        api.gather(input_tensors[0], outs if self.rank() == opts.rootRank else None, opts.rootRank, group=self._pg)
        return _done(output_tensors)

    def scatter(self, output_tensors, input_tensors, opts=ScatterOptions()):
        ins = input_tensors[0] if input_tensors else None
        api.scatter(output_tensors[0], ins if self.rank() == opts.rootRank else None, opts.rootRank, group=self._pg)
        return _done(output_tensors)

    def alltoall_base(self, output, input, output_split_sizes, input_split_sizes, opts=AllToAllOptions()):
        api.all_to_all_single(output, input, output_split_sizes or None, input_split_sizes or None, group=self._pg)
        return _done(output)

    def send(self, tensors, dst, tag):
        for t in tensors:
            api.send(t, dst, group=self._pg)
        return _done(tensors)

    def recv(self, tensors, src, tag):
        for t in tensors:
            api.recv(t, src, group=self._pg)
        return _done(tensors)

    def barrier(self, opts=BarrierOptions()):
        api.barrier(group=self._pg)
        return _done()

    def shutdown(self):
        self._pg.shutdown()


def _create(prefix_store, rank, world_size, timeout):
    return PDEProcessGroup(prefix_store, rank, world_size, timeout)


if "pde" not in tdist.Backend.backend_list:
    tdist.Backend.register_backend("pde", _create, devices=["cpu", "cuda"])
