"""``torch.distributed``-compatible process-group API over the framework's native runtime.

The reference uses exactly this surface (/root/reference/toy/main.py:16-33,
/root/reference/mnist/main.py:122-127,198-204): ``init_process_group(backend, init_method, rank,
world_size)``, ``new_group(ranks)``, ``all_reduce(tensor, op=reduce_op.SUM, group)``,
``get_world_size()`` and (through ``DistributedSampler``) ``get_rank()``.  We provide that and the
rest of the usual collective set, re-implemented MI355X-first:

* rendezvous: the framework's C++ TCP store (``csrc/runtime/store.cpp``), ``tcp://host:port`` or
  ``env://`` (MASTER_ADDR/MASTER_PORT/RANK/WORLD_SIZE).  Under ``torchrun`` the launcher already
  owns MASTER_PORT, so rank 0 starts our store on an ephemeral port and publishes it through the
  launcher's store.
* GPU tensors: RCCL communicators (``csrc/runtime/rccl_comm.cpp``) on a dedicated HIP stream per
  group, ordered against the caller's stream with events (no host synchronisation); one rank per GPU
  (``LOCAL_RANK``).  ``new_group`` splits the communicator (``ncclCommSplit``).
* CPU tensors: the C++ host TCP collectives (``csrc/runtime/hostcomm.cpp``); every group has one,
  whatever the backend string, so control-plane tensors (timings, flags) always work.
* ``backend='nccl'``/``'rccl'`` enables the RCCL path; ``'gloo'``/``'host'`` is host-only (GPU
  tensors are staged through host memory, as gloo does).
"""
from __future__ import annotations

import datetime
import enum
import os
import threading
import warnings
from typing import List, Optional

import torch

from .._ext import runtime

DEFAULT_TIMEOUT = datetime.timedelta(minutes=30)

# dtype codes shared with csrc/runtime/hostcomm.h (DType) and rccl_comm.cpp
_DTYPES = {
    torch.float32: 0, torch.float64: 1, torch.int32: 2, torch.int64: 3, torch.uint8: 4, torch.int8: 5,
    torch.bfloat16: 6, torch.float16: 7, torch.bool: 8,
}


class ReduceOp(enum.IntEnum):
    SUM = 0
    PRODUCT = 1
    MIN = 2
    MAX = 3
    AVG = 4
    BAND = 5
    BOR = 6
    BXOR = 7


class _DeprecatedReduceOp:
    """``dist.reduce_op`` (used by the reference, toy/main.py:20 and mnist/main.py:126): still
    accepted, warns like torch >= 1.x does."""

    def __getattr__(self, name):
        warnings.warn("`dist.reduce_op` is deprecated, please use `dist.ReduceOp` instead", FutureWarning,
                      stacklevel=2)
        return getattr(ReduceOp, name)


reduce_op = _DeprecatedReduceOp()


def _op_code(op) -> int:
    if isinstance(op, ReduceOp):
        return int(op)
    name = getattr(op, "name", None) or str(op).split(".")[-1]
    try:
        return int(ReduceOp[name.upper()])
    except KeyError as e:
        raise ValueError(f"unsupported reduce op {op!r}") from e


class Backend(str):
    NCCL = "nccl"
    RCCL = "rccl"
    GLOO = "gloo"
    HOST = "host"

    def __new__(cls, name: str):
        n = name.lower()
        if n not in ("nccl", "rccl", "gloo", "host", "cpu:gloo,cuda:nccl"):
            raise ValueError(f"unknown backend {name!r} (nccl/rccl = RCCL over xGMI, gloo/host = C++ TCP)")
        if n == "cpu:gloo,cuda:nccl":
            n = "nccl"
        return str.__new__(cls, n)

    @property
    def gpu(self) -> bool:
        return self in ("nccl", "rccl")


class GroupMember:
    NON_GROUP_MEMBER = object()
    WORLD = None


class Work:
    """Handle of an asynchronous collective (``async_op=True``)."""

    def __init__(self, native=None, event=None, keep=(), post=None, group=None):
        self._native = native
        self._event = event
        self._keep = keep
        self._post = post
        self._group = group
        self._done = False

    def wait(self, timeout=None):
        if self._group is not None:
            self._group.check_health()
        if self._done:
            return True
        if self._native is not None:
            self._native.wait()
        if self._event is not None:
            torch.cuda.current_stream().wait_event(self._event)
        if self._post is not None:
            self._post()
        self._done = True
        self._keep = ()
        return True

    def is_completed(self):
        if self._done:
            return True
        if self._native is not None:
            return self._native.is_completed()
        if self._event is not None:
            return self._event.query()
        return True

    def synchronize(self):
        self.wait()
        if self._event is not None:
            self._event.synchronize()       # returns once the watchdog has aborted a hung collective
        if self._group is not None:
            self._group.check_health()


class _DeferredP2P(Work):
    """Handle of a batched host isend/irecv: waiting starts the group's pending batch."""

    def __init__(self, group, keep):
        super().__init__(keep=keep)
        self._pg = group

    def wait(self, timeout=None):
        self._pg.p2p_flush()
        return super().wait(timeout)

    def is_completed(self):
        self._pg.p2p_flush()
        return super().is_completed()


class _Completed(Work):
    """Handle of a collective that already completed synchronously (host-staged GPU tensors).
    Not pre-marked done: a post-completion hook attached by the caller (e.g. DDP's copy-back of an
    fp32-staged bucket) still runs at wait()."""

    def __init__(self):
        super().__init__()


class ProcessGroup:
    def __init__(self, ranks: List[int], global_rank: int, backend: Backend, prefix: str, store, timeout_ms: int,
                 rccl=None, device=None):
        self.ranks = list(ranks)
        self.backend = backend
        self.prefix = prefix
        self.store = store
        self.global_rank = global_rank
        self._rank = self.ranks.index(global_rank)
        self.timeout_ms = timeout_ms
        self.host = runtime().HostComm(store, prefix, self._rank, len(self.ranks), timeout_ms)
        self.rccl = rccl
        self.device = device
        self._stream = None
        self._lock = threading.Lock()
        # failure detection: a collective still pending after the group timeout (dead / hung peer)
        # or an async RCCL error aborts the communicator; the next wait or collective raises
        self.watchdog = None
        if rccl is not None and os.environ.get("PDE_RCCL_WATCHDOG", "1") != "0":
            self.watchdog = runtime().CommWatchdog(rccl, timeout_ms)
        # host isend/irecv are batched until the first wait / is_completed, the group's next
        # collective or p2p call (host or RCCL), or destroy / shutdown: one full-duplex exchange then
        # moves them all, so a pairwise exchange larger than the socket buffers cannot deadlock (a
        # single background worker runs the group's host ops in order)
        self._p2p_pending = []
        # started exchanges and the tensors they read / write: kept alive here until the exchange
        # completes, even when the caller dropped the isend / irecv handle
        self._p2p_inflight = []

    def p2p_flush(self):
        """Start every deferred host isend/irecv as ONE exchange (in program order)."""
        self._p2p_inflight = [(n, k) for n, k in self._p2p_inflight if not n.is_completed()]
        if not self._p2p_pending:
            return
        pend, self._p2p_pending = self._p2p_pending, []
        sends = [(peer, t.data_ptr(), t.numel() * t.element_size()) for kind, peer, t, _ in pend if kind == "s"]
        recvs = [(peer, t.data_ptr(), t.numel() * t.element_size()) for kind, peer, t, _ in pend if kind == "r"]
        native = self.host.p2p(sends, recvs, True)
        self._p2p_inflight.append((native, [t for _, _, t, _ in pend]))
        for _, _, t, w in pend:
            w._native = native

    def check_health(self):
        if self.watchdog is not None:
            err = self.watchdog.error()
            if err:
                raise RuntimeError(err)

    # torch-compatible accessors
    def rank(self) -> int:
        return self._rank

    def size(self) -> int:
        return len(self.ranks)

    def group_rank(self, global_rank: int) -> int:
        return self.ranks.index(global_rank)

    @property
    def comm_stream(self) -> "torch.cuda.Stream":
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=self.device)
        return self._stream

    def _gpu_ok(self, t: torch.Tensor) -> bool:
        if not t.is_cuda:
            return False
        if self.rccl is None:
            return False
        if t.device.index != self.rccl.device:
            raise RuntimeError(f"tensor on {t.device} but this rank's communicator is on cuda:{self.rccl.device}")
        return True

    def shutdown(self):
        try:
            self.p2p_flush()          # queued host isend/irecv still go out (the worker drains its queue)
        except Exception:
            pass
        try:
            self.host.shutdown()
        except Exception:
            pass
        if self.watchdog is not None:
            self.watchdog.stop()
        if self.rccl is not None:
            try:
                self.rccl.destroy()
            except Exception:
                pass


_state = threading.local()
_WORLD: Optional[ProcessGroup] = None
_GROUPS = {}
_SERVER = None
_STORE = None
_GROUP_COUNTER = [0]
_RCCL_DEFAULT = None


def is_available() -> bool:
    return True


def is_initialized() -> bool:
    return _WORLD is not None


def _require_init():
    if _WORLD is None:
        raise RuntimeError("Default process group has not been initialized, please make sure to call "
                           "init_process_group.")


def get_default_group() -> ProcessGroup:
    _require_init()
    return _WORLD


def _group(group) -> Optional[ProcessGroup]:
    if group is None or group is GroupMember.WORLD:
        _require_init()
        return _WORLD
    if group is GroupMember.NON_GROUP_MEMBER:
        return None
    return group


def get_rank(group=None) -> int:
    g = _group(group)
    return -1 if g is None else g.rank()


def get_world_size(group=None) -> int:
    g = _group(group)
    return -1 if g is None else g.size()


def get_backend(group=None) -> str:
    g = _group(group)
    return str(g.backend)


def _parse_tcp(url: str):
    rest = url[len("tcp://"):]
    host, _, port = rest.rpartition(":")
    if not host or not port:
        raise ValueError(f"init_method {url!r} must be tcp://host:port")
    return host.strip("[]"), int(port)


def _rendezvous(init_method: Optional[str], rank: int, world: int, timeout_ms: int):
    """Returns (server or None, StoreClient)."""
    R = runtime()
    if init_method is None or init_method == "env://":
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500"))
        if os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true":
            # torchrun owns MASTER_PORT: publish our store's ephemeral port through its store
            from torch.distributed import TCPStore  # bootstrap only; all traffic uses our store

            agent = TCPStore(host, port, world, is_master=False,
                             timeout=datetime.timedelta(milliseconds=timeout_ms))
            key = f"pde/store/{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}/{_GROUP_COUNTER[0]}"
            server = None
            if rank == 0:
                server = R.StoreServer("0.0.0.0", 0)
                agent.set(key, str(server.port))
            port = int(agent.get(key).decode())
            return server, R.StoreClient(host, port, timeout_ms)
    elif init_method.startswith("tcp://"):
        host, port = _parse_tcp(init_method)
        if port == 0:
            # single-process job: the store takes an ephemeral port itself (no free-port probe that
            # another socket can take between the probe and the bind)
            if world != 1:
                raise ValueError(f"init_method {init_method!r}: port 0 needs world_size 1, got {world}")
            server = R.StoreServer("0.0.0.0", 0)
            return server, R.StoreClient(host, server.port, timeout_ms)
    else:
        raise ValueError(f"unsupported init_method {init_method!r} (use tcp://host:port or env://)")
    server = R.StoreServer("0.0.0.0", port) if rank == 0 else None
    return server, R.StoreClient(host, port, timeout_ms)


def _local_device() -> int:
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    return torch.cuda.current_device()


def init_process_group(backend: Optional[str] = None, init_method: Optional[str] = None,
                       timeout: Optional[datetime.timedelta] = None, world_size: int = -1, rank: int = -1,
                       store=None, group_name: str = "", device_id=None):
    """Initialise the default group (torch.distributed.init_process_group semantics)."""
    global _WORLD, _SERVER, _STORE, _RCCL_DEFAULT
    if _WORLD is not None:
        raise RuntimeError("trying to initialize the default process group twice!")
    if rank is None or (rank == -1 and "RANK" not in os.environ):
        raise ValueError(f"rank must be an integer. {rank}")
    if world_size is None or (world_size == -1 and "WORLD_SIZE" not in os.environ):
        raise ValueError(f"world_size must be an integer. {world_size}")
    rank = int(os.environ["RANK"]) if rank == -1 else int(rank)
    world_size = int(os.environ["WORLD_SIZE"]) if world_size == -1 else int(world_size)
    if not 0 <= rank < world_size:
        raise ValueError(f"invalid rank {rank} for world size {world_size}")
    be = Backend(backend or ("nccl" if torch.cuda.is_available() else "gloo"))
    timeout_ms = int((timeout or DEFAULT_TIMEOUT).total_seconds() * 1000)
    _SERVER, _STORE = _rendezvous(init_method, rank, world_size, timeout_ms)
    rccl = None
    dev = None
    if be.gpu:
        if not torch.cuda.is_available():
            raise RuntimeError("backend 'nccl' (RCCL) requires a GPU; use backend='gloo' on CPU")
        dev = device_id.index if isinstance(device_id, torch.device) else (
            device_id if device_id is not None else _local_device())
        torch.cuda.set_device(dev)
        rccl = _make_rccl(_STORE, "pde/pg0", rank, world_size, dev)
        _RCCL_DEFAULT = rccl
    _WORLD = ProcessGroup(list(range(world_size)), rank, be, "pde/pg0", _STORE, timeout_ms, rccl, dev)
    _GROUPS[tuple(range(world_size))] = _WORLD
    return _WORLD


def _make_rccl(store, prefix, rank, world, device):
    R = runtime()
    key = prefix + "/rccl_uid"
    if rank == 0:
        store.set(key, R.RcclComm.make_unique_id())
    uid = store.get(key)
    return R.RcclComm(uid, rank, world, device)


def new_group(ranks: Optional[List[int]] = None, timeout=None, backend=None, pg_options=None):
    """Collective over the default group (every rank calls it, in the same order).  Groups are cached
    by their rank tuple: the reference creates the same group on every toy step (toy/main.py:16)."""
    _require_init()
    world = _WORLD.size()
    ranks = sorted(set(range(world) if ranks is None else ranks))
    if any(r < 0 or r >= world for r in ranks):
        raise ValueError(f"new_group ranks {ranks} outside world of size {world}")
    key = tuple(ranks)
    if key in _GROUPS:
        g = _GROUPS[key]
        return g if _WORLD.global_rank in ranks else GroupMember.NON_GROUP_MEMBER
    _GROUP_COUNTER[0] += 1
    prefix = f"pde/grp{_GROUP_COUNTER[0]}"
    me = _WORLD.global_rank
    rccl = None
    if _WORLD.rccl is not None:
        # ncclCommSplit is collective over the parent: non-members pass NOCOLOR
        rccl = _WORLD.rccl.split(0 if me in ranks else -1, me)
    if me not in ranks:
        _GROUPS[key] = None
        return GroupMember.NON_GROUP_MEMBER
    be = Backend(backend) if backend else _WORLD.backend
    timeout_ms = int(timeout.total_seconds() * 1000) if timeout else _WORLD.timeout_ms
    g = ProcessGroup(ranks, me, be, prefix, _STORE, timeout_ms, rccl if be.gpu else None, _WORLD.device)
    _GROUPS[key] = g
    return g


def destroy_process_group(group=None):
    global _WORLD, _SERVER, _STORE, _RCCL_DEFAULT
    if group is not None and group is not GroupMember.WORLD and group is not _WORLD:
        if isinstance(group, ProcessGroup):
            group.shutdown()
            for k, v in list(_GROUPS.items()):
                if v is group:
                    del _GROUPS[k]
        return
    if _WORLD is None:
        return
    for g in set(v for v in _GROUPS.values() if v is not None):
        if g is not _WORLD:
            g.shutdown()
    try:
        _WORLD.p2p_flush()        # an un-waited isend/irecv must still reach its peer
        _WORLD.host.barrier()     # let every rank finish before the store server goes away
    except Exception:
        pass
    _WORLD.shutdown()
    _GROUPS.clear()
    _WORLD = None
    _RCCL_DEFAULT = None
    _STORE = None
    if _SERVER is not None:
        _SERVER.stop()
        _SERVER = None


# ------------------------------------------------------------------------------------------------
# collectives
# ------------------------------------------------------------------------------------------------
def _check(t: torch.Tensor):
    if not isinstance(t, torch.Tensor):
        raise TypeError("collectives take tensors")
    if not t.is_contiguous():
        raise ValueError("tensors must be contiguous")
    if t.dtype not in _DTYPES:
        raise TypeError(f"unsupported dtype {t.dtype}")


def gpu_launch(g: ProcessGroup, tensors, fn, async_op: bool, what: str = "collective"):
    """Run fn(stream_handle) on the group's comm stream, ordered after the caller's stream (the
    watchdog covers it when the group has RCCL); returns a Work (async) or joins the caller's stream."""
    g.check_health()
    g.p2p_flush()        # host isend/irecv issued before this collective start now (asynchronously)
    cur = torch.cuda.current_stream(g.device)
    cs = g.comm_stream
    cs.wait_stream(cur)
    with torch.cuda.stream(cs):
        fn(cs.cuda_stream)
    if g.watchdog is not None:
        g.watchdog.watch(cs.cuda_stream, what)
    for t in tensors:
        t.record_stream(cs)
    ev = torch.cuda.Event()
    ev.record(cs)
    if async_op:
        return Work(event=ev, keep=tuple(tensors), group=g)
    cur.wait_event(ev)
    return None


def _host(g: ProcessGroup):
    """The group's host collective, after any deferred point-to-point batch (program order)."""
    g.p2p_flush()
    return g.host


def _host_staged(tensors, fn):
    """GPU tensors on a host-only group: stage through CPU (gloo semantics)."""
    cpu = [t.detach().cpu() for t in tensors]
    fn(cpu)
    for t, c in zip(tensors, cpu):
        t.copy_(c)


def all_reduce(tensor: torch.Tensor, op=ReduceOp.SUM, group=None, async_op: bool = False):
    g = _group(group)
    if g is None:
        return None
    _check(tensor)
    code, dt, n = _op_code(op), _DTYPES[tensor.dtype], tensor.numel()
    if g._gpu_ok(tensor) and code <= 4:      # RCCL has no bitwise reductions
        return gpu_launch(g, [tensor], lambda s: g.rccl.all_reduce(tensor.data_ptr(), tensor.data_ptr(), n, dt,
                                                                     code, s), async_op)
    if tensor.is_cuda:
        _host_staged([tensor], lambda c: _host(g).allreduce(c[0].data_ptr(), n, dt, code))
        return _Completed() if async_op else None
    w = _host(g).allreduce(tensor.data_ptr(), n, dt, code, async_op)
    return Work(native=w, keep=(tensor,)) if async_op else None


def broadcast(tensor: torch.Tensor, src: int = 0, group=None, async_op: bool = False):
    g = _group(group)
    if g is None:
        return None
    _check(tensor)
    root = g.group_rank(src)
    if g._gpu_ok(tensor):
        return gpu_launch(g, [tensor], lambda s: g.rccl.broadcast(tensor.data_ptr(), tensor.data_ptr(),
                                                                    tensor.numel(), _DTYPES[tensor.dtype], root, s),
                           async_op)
    if tensor.is_cuda:
        _host_staged([tensor], lambda c: _host(g).broadcast(c[0].data_ptr(), c[0].numel() * c[0].element_size(), root))
        return _Completed() if async_op else None
    w = _host(g).broadcast(tensor.data_ptr(), tensor.numel() * tensor.element_size(), root, async_op)
    return Work(native=w, keep=(tensor,)) if async_op else None


def all_gather_into_tensor(output_tensor: torch.Tensor, input_tensor: torch.Tensor, group=None,
                           async_op: bool = False):
    g = _group(group)
    if g is None:
        return None
    _check(output_tensor)
    _check(input_tensor)
    if output_tensor.numel() != input_tensor.numel() * g.size():
        raise ValueError("output must hold world_size x input elements")
    if g._gpu_ok(input_tensor):
        return gpu_launch(g, [output_tensor, input_tensor],
                           lambda s: g.rccl.all_gather(input_tensor.data_ptr(), output_tensor.data_ptr(),
                                                       input_tensor.numel(), _DTYPES[input_tensor.dtype], s),
                           async_op)
    if input_tensor.is_cuda:
        def f(c):
            _host(g).allgather(c[1].data_ptr(), c[0].data_ptr(), c[1].numel() * c[1].element_size())
        _host_staged([output_tensor, input_tensor], f)
        return _Completed() if async_op else None
    w = _host(g).allgather(input_tensor.data_ptr(), output_tensor.data_ptr(),
                         input_tensor.numel() * input_tensor.element_size(), async_op)
    return Work(native=w, keep=(output_tensor, input_tensor)) if async_op else None


def all_gather(tensor_list: List[torch.Tensor], tensor: torch.Tensor, group=None, async_op: bool = False):
    g = _group(group)
    if g is None:
        return None
    flat = torch.empty((g.size(),) + tuple(tensor.shape), dtype=tensor.dtype, device=tensor.device)
    w = all_gather_into_tensor(flat, tensor.contiguous(), group=g, async_op=async_op)

    def post():
        for i, t in enumerate(tensor_list):
            t.copy_(flat[i])

    if async_op:
        w._post = post
        return w
    post()
    return None


def reduce_scatter_tensor(output: torch.Tensor, input: torch.Tensor, op=ReduceOp.SUM, group=None,
                          async_op: bool = False):
    g = _group(group)
    if g is None:
        return None
    _check(output)
    _check(input)
    if input.numel() != output.numel() * g.size():
        raise ValueError("input must hold world_size x output elements")
    code, dt = _op_code(op), _DTYPES[input.dtype]
    if g._gpu_ok(input) and code <= 4:
        return gpu_launch(g, [output, input], lambda s: g.rccl.reduce_scatter(input.data_ptr(), output.data_ptr(),
                                                                               output.numel(), dt, code, s), async_op)
    if input.is_cuda:
        _host_staged([output, input], lambda c: _host(g).reduce_scatter(c[1].data_ptr(), c[0].data_ptr(),
                                                                      c[0].numel(), dt, code))
        return _Completed() if async_op else None
    w = _host(g).reduce_scatter(input.data_ptr(), output.data_ptr(), output.numel(), dt, code, async_op)
    return Work(native=w, keep=(output, input)) if async_op else None


def reduce_scatter(output: torch.Tensor, input_list: List[torch.Tensor], op=ReduceOp.SUM, group=None,
                   async_op: bool = False):
    return reduce_scatter_tensor(output, torch.cat([t.reshape(-1) for t in input_list]), op, group, async_op)


def reduce(tensor: torch.Tensor, dst: int = 0, op=ReduceOp.SUM, group=None, async_op: bool = False):
    g = _group(group)
    if g is None:
        return None
    _check(tensor)
    root, code, dt, n = g.group_rank(dst), _op_code(op), _DTYPES[tensor.dtype], tensor.numel()
    if g._gpu_ok(tensor) and code <= 4:
        return gpu_launch(g, [tensor], lambda s: g.rccl.reduce(tensor.data_ptr(), tensor.data_ptr(), n, dt, code,
                                                                 root, s), async_op)
    if tensor.is_cuda:
        _host_staged([tensor], lambda c: _host(g).reduce(c[0].data_ptr(), n, dt, code, root))
        return _Completed() if async_op else None
    w = _host(g).reduce(tensor.data_ptr(), n, dt, code, root, async_op)
    return Work(native=w, keep=(tensor,)) if async_op else None


def gather(tensor: torch.Tensor, gather_list: Optional[List[torch.Tensor]] = None, dst: int = 0, group=None,
           async_op: bool = False):
    g = _group(group)
    if g is None:
        return None
    out = torch.empty((g.size(),) + tuple(tensor.shape), dtype=tensor.dtype, device=tensor.device)
    all_gather_into_tensor(out, tensor.contiguous(), group=g)   # simple and correct for small control data
    if g.global_rank == dst and gather_list is not None:
        for i, t in enumerate(gather_list):
            t.copy_(out[i])
    return _Completed() if async_op else None


def scatter(tensor: torch.Tensor, scatter_list: Optional[List[torch.Tensor]] = None, src: int = 0, group=None,
            async_op: bool = False):
    g = _group(group)
    if g is None:
        return None
    root = g.group_rank(src)
    if tensor.is_cuda and g._gpu_ok(tensor):
        buf = (torch.stack([t.reshape(tensor.shape) for t in scatter_list]) if g.rank() == root
               else torch.empty((g.size(),) + tuple(tensor.shape), dtype=tensor.dtype, device=tensor.device))
        broadcast(buf, src, group=g)
        tensor.copy_(buf[g.rank()])
        return _Completed() if async_op else None
    cpu_in = (torch.stack([t.detach().cpu().reshape(tensor.shape) for t in scatter_list]).contiguous()
              if g.rank() == root else torch.empty(0, dtype=tensor.dtype))
    out = torch.empty(tensor.shape, dtype=tensor.dtype).contiguous()
    _host(g).scatter(cpu_in.data_ptr() if g.rank() == root else 0, out.data_ptr(), out.numel() * out.element_size(),
                   root)
    tensor.copy_(out)
    return _Completed() if async_op else None


def all_to_all_single(output: torch.Tensor, input: torch.Tensor, output_split_sizes=None, input_split_sizes=None,
                      group=None, async_op: bool = False):
    g = _group(group)
    if g is None:
        return None
    if output_split_sizes is not None or input_split_sizes is not None:
        raise NotImplementedError("uneven all_to_all_single splits")
    _check(output)
    _check(input)
    per = input.numel() // g.size()
    if g._gpu_ok(input):
        return gpu_launch(g, [output, input], lambda s: g.rccl.all_to_all(input.data_ptr(), output.data_ptr(), per,
                                                                           _DTYPES[input.dtype], s), async_op)
    if input.is_cuda:
        _host_staged([output, input], lambda c: _host(g).alltoall(c[1].data_ptr(), c[0].data_ptr(),
                                                                per * c[1].element_size()))
        return _Completed() if async_op else None
    w = _host(g).alltoall(input.data_ptr(), output.data_ptr(), per * input.element_size(), async_op)
    return Work(native=w, keep=(output, input)) if async_op else None


def send(tensor: torch.Tensor, dst: int, group=None, tag: int = 0):
    g = _group(group)
    _check(tensor)
    peer = g.group_rank(dst)
    if g._gpu_ok(tensor):
        gpu_launch(g, [tensor], lambda s: g.rccl.send(tensor.data_ptr(), tensor.numel(), _DTYPES[tensor.dtype],
                                                       peer, s), False)
        return
    t = tensor.detach().cpu().contiguous() if tensor.is_cuda else tensor
    _host(g).send(t.data_ptr(), t.numel() * t.element_size(), peer)


def recv(tensor: torch.Tensor, src: Optional[int] = None, group=None, tag: int = 0):
    g = _group(group)
    _check(tensor)
    if src is None:
        raise NotImplementedError("recv from any source")
    peer = g.group_rank(src)
    if g._gpu_ok(tensor):
        gpu_launch(g, [tensor], lambda s: g.rccl.recv(tensor.data_ptr(), tensor.numel(), _DTYPES[tensor.dtype],
                                                       peer, s), False)
        return src
    if tensor.is_cuda:
        c = torch.empty(tensor.shape, dtype=tensor.dtype)
        _host(g).recv(c.data_ptr(), c.numel() * c.element_size(), peer)
        tensor.copy_(c)
    else:
        _host(g).recv(tensor.data_ptr(), tensor.numel() * tensor.element_size(), peer)
    return src


def _defer(g: ProcessGroup, kind: str, tensor: torch.Tensor, peer: int) -> Work:
    _check(tensor)
    w = _DeferredP2P(g, keep=(tensor,))
    g._p2p_pending.append((kind, g.group_rank(peer), tensor, w))
    return w


def isend(tensor: torch.Tensor, dst: int, group=None, tag: int = 0):
    g = _group(group)
    if tensor.is_cuda:
        send(tensor, dst, g, tag)
        return _Completed()
    return _defer(g, "s", tensor, dst)


def irecv(tensor: torch.Tensor, src: Optional[int] = None, group=None, tag: int = 0):
    g = _group(group)
    if tensor.is_cuda or src is None:
        recv(tensor, src, g, tag)
        return _Completed()
    return _defer(g, "r", tensor, src)


class P2POp:
    """One point-to-point op for ``batch_isend_irecv`` (``op`` is ``isend`` or ``irecv``)."""

    def __init__(self, op, tensor: torch.Tensor, peer: int, group=None, tag: int = 0):
        if op not in (isend, irecv):
            raise ValueError("P2POp op must be dist.isend or dist.irecv")
        self.op, self.tensor, self.peer, self.group, self.tag = op, tensor, peer, group, tag


def batch_isend_irecv(p2p_op_list: List[P2POp]) -> List[Work]:
    """Issue a set of sends/receives together.  GPU: one ``ncclGroupStart/End`` on the comm stream, so
    any send/recv pattern (rings, exchanges, all-to-all by hand) progresses without deadlock.  Host:
    one full-duplex socket exchange over all of the batch's sends and receives."""
    if not p2p_op_list:
        return []
    g = _group(p2p_op_list[0].group)
    if any(_group(o.group) is not g for o in p2p_op_list):
        raise ValueError("batch_isend_irecv: all ops must use the same group")
    for o in p2p_op_list:
        _check(o.tensor)
    if all(g._gpu_ok(o.tensor) for o in p2p_op_list):
        def fn(stream):
            g.rccl.group_start()
            try:
                for o in p2p_op_list:
                    t = o.tensor
                    f = g.rccl.send if o.op is isend else g.rccl.recv
                    f(t.data_ptr(), t.numel(), _DTYPES[t.dtype], g.group_rank(o.peer), stream)
            finally:
                g.rccl.group_end()
        w = gpu_launch(g, [o.tensor for o in p2p_op_list], fn, True)
        return [w]
    # host: every send and receive of the batch in ONE full-duplex exchange (GPU tensors staged)
    staged = []
    works = []
    for o in p2p_op_list:
        t = o.tensor
        if t.is_cuda:
            c = t.detach().cpu().contiguous() if o.op is isend else torch.empty(t.shape, dtype=t.dtype)
            staged.append((o, c))
            t = c
        works.append(_defer(g, "s" if o.op is isend else "r", t, o.peer))
    g.p2p_flush()
    if staged:
        for w in works:
            w.wait()
        for o, c in staged:
            if o.op is irecv:
                o.tensor.copy_(c)
    return works


def barrier(group=None, async_op: bool = False, device_ids=None):
    g = _group(group)
    if g is None:
        return None
    if g.rccl is not None and torch.cuda.is_available():
        torch.cuda.synchronize(g.device)          # device work issued before the barrier is done
    w = _host(g).barrier(async_op)
    return Work(native=w) if async_op else None


# ------------------------------------------------------------------------------------------------
# framework helpers
# ------------------------------------------------------------------------------------------------
class EngineComm:
    """Comm handle for the fused training engines: SUM all-reduce of a flat buffer enqueued on the
    CURRENT stream (the engine puts it on its comm stream and captures it in hipGraphs).

    ``enable_peer(sizes)`` adds the xGMI peer all-reduce (``dist/peer.py``) for small buffers and
    times it against RCCL at exactly those sizes; each size then takes the faster route.  A group
    without RCCL (gloo, e.g. several ranks sharing one GPU in tests) routes everything to the peer
    kernel."""

    def __init__(self, group: ProcessGroup, allow_host_only: bool = False):
        if group.rccl is None and not allow_host_only:
            raise RuntimeError("engine comm needs an RCCL (backend='nccl') process group")
        self.group = group
        self.world_size = group.size()
        self.rank = group.rank()
        self.peer = None
        self.peer_reason = ""
        self.peer_inplace = False
        self.routes = {}
        self.timings = {}

    def _rccl(self, t: torch.Tensor, op=ReduceOp.SUM):
        self.group.rccl.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _DTYPES[t.dtype], _op_code(op),
                                   torch.cuda.current_stream(t.device).cuda_stream)

    def enable_peer(self, sizes, device, dtype=torch.float32, capacity_bytes: Optional[int] = None, tune=True,
                    inplace: Optional[torch.Tensor] = None, bufs: Optional[dict] = None):
        """Collective.  Returns the chosen route per size ({numel: 'rccl'|'peer1'|'peer2'}).
        ``inplace``: a persistent fp32 buffer (the engine's flat gradients) to register, so the peer
        routes of any range of it run in place (no stage copy; ``PDE_PEER_INPLACE=0`` disables);
        ``bufs``: {numel: tensor} -- the tensors the routes will run on, timed instead of scratch ones."""
        from .peer import PeerAllReduce, tune_routes
        sizes = sorted({int(n) for n in sizes})
        esize = torch.tensor([], dtype=dtype).element_size()
        cap = capacity_bytes or max(sizes) * esize
        self.peer_inplace = False
        if os.environ.get("PDE_PEER_ALLREDUCE", "1") != "0":
            self.peer = PeerAllReduce(self.group, torch.device(device), cap)
            if not self.peer.ok:
                self.peer_reason = self.peer.reason
                self.peer = None
        else:
            self.peer_reason = "disabled by PDE_PEER_ALLREDUCE=0"
        if self.peer is not None and inplace is not None and os.environ.get("PDE_PEER_INPLACE", "1") != "0":
            self.peer_inplace = self.peer.register(inplace)
            if not self.peer_inplace:
                self.peer_reason = self.peer.reg_reason
        rccl_fn = self._rccl if self.group.rccl is not None else None
        if tune:
            self.routes, self.timings = tune_routes(self.group, self.peer, rccl_fn, sizes, device, dtype, bufs=bufs)
        else:
            self.routes = {n: ("peer2" if self.peer is not None else "rccl") for n in sizes}
        return self.routes

    def route(self, t: torch.Tensor) -> str:
        r = self.routes.get(t.numel())
        if r is None:
            r = "rccl" if self.group.rccl is not None or self.peer is None else "peer2"
        if r != "rccl" and not (self.peer is not None and self.peer.supports(t)):
            r = "rccl"
        if r == "rccl" and self.group.rccl is None:
            raise RuntimeError("no RCCL communicator and the peer all-reduce cannot take this buffer")
        return r

    def all_reduce_(self, t: torch.Tensor, op=ReduceOp.SUM):
        r = self.route(t) if _op_code(op) in (0, 4) else "rccl"
        if r == "rccl":
            self._rccl(t, op)
        else:
            self.peer.all_reduce_(t, r, scale=(1.0 / self.world_size) if _op_code(op) == 4 else 1.0)

    def health(self) -> str:
        """'' if healthy, else a description of the failure (peer barrier time-outs, RCCL errors)."""
        if self.peer is not None and self.peer.error():
            return f"peer all-reduce: {self.peer.error()} barrier time-out(s)"
        if self.group.watchdog is not None:
            return self.group.watchdog.error()
        return ""


def engine_comm(group=None, allow_host_only: bool = False) -> EngineComm:
    return EngineComm(_group(group), allow_host_only)


@torch.no_grad()
def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None, buffers: bool = True):
    """Make every rank's replica identical (DDP semantics; the reference never does this, survey Q2)."""
    tensors = [p.data for p in module.parameters()]
    if buffers:
        tensors += [b for b in module.buffers()]
    broadcast_coalesced(tensors, src, group)


@torch.no_grad()
def broadcast_coalesced(tensors, src: int = 0, group=None):
    """Broadcast a list of tensors with ONE collective per (device, dtype): flatten, broadcast, scatter
    back (torch DDP's ``_broadcast_coalesced``)."""
    g = _group(group)
    if g is None or g.size() == 1:
        return
    by_dev = {}
    for t in tensors:
        by_dev.setdefault((t.device, t.dtype), []).append(t)
    for (_, _), ts in by_dev.items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        broadcast(flat, src, group=g)
        o = 0
        for t in ts:
            t.copy_(flat[o:o + t.numel()].view_as(t))
            o += t.numel()
