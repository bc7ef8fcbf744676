"""xGMI peer all-reduce for small, latency-bound buffers (``csrc/runtime/peer_allreduce.hip``).

The reference averages gradients with one blocking all-reduce per parameter
(/root/reference/mnist/main.py:122-127); the framework packs them into two flat buckets
(1.62 MB + 0.10 MB for the toy CNN).  At that size a ring all-reduce over 8 GPUs is dominated by
its 2·(W-1) dependent hops, so for small buckets every rank instead reads its peers' staged data
directly over the 7 point-to-point xGMI links (one-shot: one barrier; two-shot: reduce-scatter +
all-gather through peer memory, two barriers).  Large buckets (ResNet-18 / GPT-2) stay on RCCL.

``PeerAllReduce(group)`` is collective over a process group: every rank allocates a flag region
(uncached) and a data region (PDE_PEER_UNCACHED=1: uncached too), exchanges their IPC handles through the group's TCP store, maps every peer's region,
and then runs a self-test of both algorithms (f32 and bf16, ragged sizes) against the exact
answer.  Any failure on any rank (IPC unsupported, wrong sums, a barrier time-out) disables the
path on every rank and the caller keeps using RCCL.

``PDE_PEER_FORCE_FAIL=<rank>[,<rank>...]`` makes those ranks fail the set-up (failure-path tests:
every rank must then agree on RCCL only).  ``PDE_PEER_DEBUG_STALE=<rank>`` makes that rank skip
staging one self-test call (a stale stage buffer): the self-test must then disable the path.

``register(tensor)`` (collective) IPC-maps a persistent fp32 buffer of every rank (the engines' flat
gradient buffer): an all-reduce of any range of it then runs IN PLACE -- the peers' gradients are read
where the backward left them, with no stage copy and no L2 write-back / invalidate fences (only flag
barriers; ``peer_allreduce.h``).  Registration runs its own self-test of both algorithms on the
buffer (its contents are clobbered, then zeroed) and is voted on like the set-up.

``tune_routes`` times RCCL against the one-/two-shot peer kernels at the sizes an engine will use
(max over ranks, so every rank takes the same decision) and returns the fastest per size.
"""
from __future__ import annotations

import os
import sys
from typing import Dict, Iterable, Optional

import torch

from .._ext import runtime

ONE_SHOT, TWO_SHOT, RCCL = "peer1", "peer2", "rccl"
_ALGO = {ONE_SHOT: 1, TWO_SHOT: 2}
_SEQ = [0]


def _host_allreduce_min(group, value: int) -> int:
    t = torch.tensor([int(value)], dtype=torch.int64)
    group.host.allreduce(t.data_ptr(), 1, 3, 2)     # int64, MIN
    return int(t.item())


_REG_DTYPES = (torch.float32, torch.bfloat16)
_ONE_SHOT_MAX_BYTES = 256 * 512 * 4 * 16        # in-place one-shot: <= 4 vectors per thread, 256 blocks


def _host_allreduce_max_f64(group, vals) -> list:
    t = torch.tensor(list(vals), dtype=torch.float64)
    group.host.allreduce(t.data_ptr(), t.numel(), 1, 3)   # float64, MAX
    return t.tolist()


def _device_uuid(device: torch.device) -> str:
    try:
        return str(torch.cuda.get_device_properties(device).uuid)
    except Exception:   # noqa: BLE001 - older torch: fall back to the index (the rank's own view)
        return f"index-{torch.device(device).index}"


class PeerAllReduce:
    """Collective constructor; see the module docstring.  ``ok`` says whether the path is usable."""

    def __init__(self, group, device: torch.device, capacity_bytes: int, timeout_ms: Optional[int] = None,
                 self_test: bool = True):
        # barrier time-out: a dead / hung peer latches an error instead of hanging (PDE_PEER_TIMEOUT_MS)
        if timeout_ms is None:
            timeout_ms = int(os.environ.get("PDE_PEER_TIMEOUT_MS", "10000"))
        self.group = group
        self.device = torch.device(device)
        self.rank, self.world = group.rank(), group.size()
        self.native = None
        self.ok = False
        self.reason = ""
        self.reg_reason = ""
        self._regs = []          # (data_ptr, numel, registration id, tensor kept alive)
        self.shared = 1
        _SEQ[0] += 1
        key = f"{group.prefix}/peer_ar/{_SEQ[0]}"
        err = ""
        try:
            if str(self.rank) in os.environ.get("PDE_PEER_FORCE_FAIL", "").split(","):
                raise RuntimeError("forced by PDE_PEER_FORCE_FAIL")      # failure-path tests
            self.native = runtime().PeerAllReduce(self.rank, self.world, self.device.index, int(capacity_bytes),
                                                  os.environ.get("PDE_PEER_UNCACHED", "0") == "1")
            self.native.set_timeout_ms(int(timeout_ms))
            group.store.set(f"{key}/h{self.rank}", self.native.handle())
            group.store.set(f"{key}/dev{self.rank}", str(self.device.index).encode())
            group.store.set(f"{key}/uuid{self.rank}", _device_uuid(self.device).encode())
        except Exception as e:   # noqa: BLE001 - any failure means "no peer path"
            err = f"setup: {e}"
            group.store.set(f"{key}/h{self.rank}", b"")
            group.store.set(f"{key}/dev{self.rank}", b"-1")
            group.store.set(f"{key}/uuid{self.rank}", f"none-{self.rank}".encode())
        handles = [group.store.get(f"{key}/h{r}") for r in range(self.world)]
        devs = [int(group.store.get(f"{key}/dev{r}")) for r in range(self.world)]
        uuids = [group.store.get(f"{key}/uuid{r}").decode() for r in range(self.world)]
        if not err:
            try:
                if any(len(h) == 0 for h in handles):
                    raise RuntimeError("a peer failed to create its region")
                me = self.device.index
                for d in set(devs):
                    if d != me and not torch.cuda.can_device_access_peer(me, d):
                        raise RuntimeError(f"cuda:{me} cannot access peer cuda:{d}")
                self.native.open(handles)
                # ranks time-sharing this GPU (1 on a real node), by physical device (a per-rank
                # HIP_VISIBLE_DEVICES makes every rank's index 0)
                self.shared = uuids.count(uuids[self.rank])
                if self.shared > 1:
                    # every sharing rank's spinning grid must be co-resident (else a rank's kernel waits
                    # for CUs that another rank's blocks hold while they wait for it: a deadlock until
                    # the barrier time-out -- seen with 8 ranks on one GPU)
                    self.native.set_max_blocks(max(1, min(64, 256 // self.shared)))
                    self.native.set_ip_block_cap(max(1, 256 // self.shared))
            except Exception as e:   # noqa: BLE001
                err = f"open: {e}"
        ok = _host_allreduce_min(group, 0 if err else 1)
        group.host.barrier()
        if ok and self_test:
            # first launches load the code object in every process (slow when ranks share a GPU):
            # generous barrier time-out for the self-test, the steady-state one afterwards
            self.native.set_timeout_ms(max(int(timeout_ms), 60000))
            try:
                self._self_test()
            except Exception as e:   # noqa: BLE001
                err = f"self-test: {e}"
            self.native.set_timeout_ms(int(timeout_ms))
            ok = _host_allreduce_min(group, 0 if err else 1)
        self.ok = bool(ok)
        self.reason = err or ("" if ok else "disabled by a peer rank")
        if not self.ok:
            print(f"[rank {self.rank}] xGMI peer all-reduce disabled: {self.reason}", file=sys.stderr, flush=True)
        if not self.ok and self.native is not None:
            try:
                self.native.close()
            except Exception:   # noqa: BLE001
                pass
            self.native = None

    def register(self, t: torch.Tensor, self_test: bool = True) -> bool:
        """Collective: map every rank's ``t`` (contiguous fp32 or bf16, the same size on every rank) so that
        ``all_reduce_`` of any 16-byte-aligned range of it runs in place.  False (on every rank) if any
        rank failed; the staged path stays available either way."""
        if not self.ok:
            return False
        _SEQ[0] += 1
        key = f"{self.group.prefix}/peer_reg/{_SEQ[0]}"
        err, rid = "", -1
        try:
            if t.dtype not in _REG_DTYPES or not t.is_contiguous() or t.device != self.device:
                raise ValueError("registered buffers are contiguous fp32 / bf16 tensors on the rank's device")
            rid, h = self.native.register_buffer(t.data_ptr(), t.numel() * t.element_size())
            self.group.store.set(f"{key}/h{self.rank}", h)
        except Exception as e:   # noqa: BLE001
            err = f"register: {e}"
            self.group.store.set(f"{key}/h{self.rank}", b"")
        hs = [self.group.store.get(f"{key}/h{r}") for r in range(self.world)]
        if not err:
            try:
                if any(len(h) == 0 for h in hs):
                    raise RuntimeError("a peer failed to register its buffer")
                self.native.open_registered(rid, hs)
            except Exception as e:   # noqa: BLE001
                err = f"open registered: {e}"
        ok = _host_allreduce_min(self.group, 0 if err else 1)
        if ok and self_test:
            try:
                self._self_test_registered(t, rid)
            except Exception as e:   # noqa: BLE001
                err = f"registered self-test: {e}"
            ok = _host_allreduce_min(self.group, 0 if err else 1)
        if not ok:
            print(f"[rank {self.rank}] in-place peer all-reduce disabled: {err or 'disabled by a peer rank'}",
                  file=sys.stderr, flush=True)
            self.reg_reason = err or "disabled by a peer rank"
            return False
        self._regs.append((t.data_ptr(), t.numel(), rid, t))
        return True

    def registered_range(self, t: torch.Tensor):
        """(registration id, element offset) if ``t`` is a 16-byte aligned range of a registered buffer
        of its dtype, else None."""
        if t.dtype not in _REG_DTYPES or not t.is_contiguous():
            return None
        p, esz = t.data_ptr(), t.element_size()
        for base, n, rid, buf in self._regs:
            if buf.dtype == t.dtype and base <= p and p + t.numel() * esz <= base + n * esz and (p - base) % 16 == 0:
                return rid, (p - base) // esz
        return None

    def _self_test_registered(self, buf: torch.Tensor, rid: int):
        W, r = self.world, self.rank
        n_all = buf.numel()
        call = [0]

        esz, per = buf.element_size(), 16 // buf.element_size()

        def data(n, rank, c):   # small integers: every sum is exact in bf16 too
            i = torch.arange(n, device=self.device, dtype=torch.int64)
            return (((i * 7 + c * 13 + rank * 5) % 17) - 8).to(buf.dtype)

        s = torch.cuda.current_stream(self.device)
        # the test runs on the live buffer (the registration covers exactly it): whatever it holds --
        # e.g. gradients accumulated before a DDP wrapper was built -- is restored afterwards
        saved = buf.detach().clone()
        for n in sorted({1, 5, 4099, min(n_all, 70001), n_all - (n_all % per)}):
            if n <= 0 or n > n_all:
                continue
            for algo in (1, 2):
                if algo == 1 and n * esz > _ONE_SHOT_MAX_BYTES:
                    continue
                for off in (0, per * ((n_all - n) // (2 * per))):      # two offsets inside the buffer
                    c = call[0]
                    call[0] += 1
                    buf[off:off + n].copy_(data(n, r, c))
                    self.native.all_reduce_registered(rid, off, n, esz, 1.0, algo, s.cuda_stream)
                    torch.cuda.synchronize(self.device)
                    if self.error():
                        raise RuntimeError(f"barrier time-out (algo {algo}, n={n}, off={off})")
                    want = sum(data(n, q, c) for q in range(W))
                    if not torch.equal(buf[off:off + n], want):
                        bad = int((buf[off:off + n] != want).sum())
                        raise RuntimeError(f"algo {algo} n={n} off={off} call {c}: {bad} wrong elements")
        buf.copy_(saved)
        torch.cuda.synchronize(self.device)
        del saved

    @property
    def capacity_bytes(self) -> int:
        return self.native.capacity_bytes if self.native is not None else 0

    def supports(self, t: torch.Tensor) -> bool:
        if self.ok and self.registered_range(t) is not None:
            return True
        return (self.ok and t.is_cuda and t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous()
                and t.numel() * t.element_size() <= self.capacity_bytes and t.data_ptr() % 16 == 0)

    def all_reduce_(self, t: torch.Tensor, algo: str = "auto", scale: float = 1.0, stream=None):
        """In-place SUM (times ``scale``) on ``stream`` (default: the current stream): straight on the
        peers' buffers when ``t`` lies in a registered buffer, else through the staged regions."""
        s = stream if stream is not None else torch.cuda.current_stream(t.device)
        a = _ALGO.get(algo, 0)
        reg = self.registered_range(t)
        if reg is not None:
            if a == 1 and t.numel() * t.element_size() > _ONE_SHOT_MAX_BYTES:   # two-shot in place
                a = 2
            self.native.all_reduce_registered(reg[0], reg[1], t.numel(), t.element_size(), float(scale), a,
                                              s.cuda_stream)
            return
        fn = self.native.all_reduce_f32 if t.dtype == torch.float32 else self.native.all_reduce_bf16
        fn(t.data_ptr(), t.data_ptr(), t.numel(), float(scale), a, s.cuda_stream)

    def error(self) -> int:
        return int(self.native.error()) if self.native is not None else 0

    def error_async(self) -> int:
        """Time-out latch as mirrored to host memory by the kernels: no device synchronisation (a call
        still queued has not reported yet).  After a time-out every call writes NaN, never a partial sum."""
        return int(self.native.error_async()) if self.native is not None else 0

    def _self_test(self):
        """Both algorithms of the host kernel (f32 and bf16, ragged sizes) and the device-side protocol
        of pde_peer_dev.h (f32, one- and two-shot), against the exact answer.  Every call gets data of
        its own (a per-call counter is mixed into every element), and a run of consecutive calls
        visits both stage parities several times: a rank that reads a peer's stage buffer as it was
        one or two calls ago gets a wrong sum (``PDE_PEER_DEBUG_STALE=<rank>`` injects exactly that:
        the rank skips staging one call).  Values are small integers, so every sum is exact in bf16."""
        W, r = self.world, self.rank
        cap_el = self.capacity_bytes // 4
        sizes = sorted({1, 3, 5, 1000, 4099, min(cap_el, 70001), cap_el - 3})
        call = [0]

        def data(n, rank, c):
            i = torch.arange(n, device=self.device, dtype=torch.int64)
            return (((i * 7 + c * 13 + rank * 5) % 17) - 8).to(torch.float32)

        def check(x, n, dtype, what):
            c = call[0]
            call[0] += 1
            torch.cuda.synchronize(self.device)
            if self.error():
                raise RuntimeError(f"barrier time-out during self-test ({what} {dtype} n={n} call {c})")
            want = sum(data(n, q, c) for q in range(W)).to(dtype)
            if not torch.equal(x, want):
                bad = int((x != want).sum())
                raise RuntimeError(f"{what} {dtype} n={n} call {c}: {bad} wrong elements")

        stale = str(r) in os.environ.get("PDE_PEER_DEBUG_STALE", "").split(",")
        for dtype in (torch.float32, torch.bfloat16):
            for n in sizes:
                if n <= 0 or n * (4 if dtype == torch.float32 else 2) > self.capacity_bytes:
                    continue
                reps = 8 if n == 4099 else 2          # 8 consecutive calls: 4 per stage parity
                for algo in (ONE_SHOT, TWO_SHOT):
                    for _ in range(reps):
                        if stale and call[0] == 5:
                            self.native.debug_skip_stage(1)
                        x = data(n, r, call[0]).to(dtype)
                        self.all_reduce_(x, algo)
                        check(x, n, dtype, algo)
        s = torch.cuda.current_stream(self.device)
        for n in (5, 4099, min(cap_el, 70001)):
            for two in (0, 1):
                for _ in range(8):
                    x = data(n, r, call[0])
                    self.native.device_probe_f32(x.data_ptr(), x.data_ptr(), n, 1.0, two, s.cuda_stream)
                    check(x, n, torch.float32, "device-path two-shot" if two else "device-path one-shot")
        if self.error():
            raise RuntimeError("barrier time-out during self-test")

    def close(self):
        if self.native is not None:
            self.native.close()
            self.native = None
            self.ok = False


def _time_calls(fn, iters: int, device, group=None) -> float:
    """GPU time per call: ``iters`` calls captured in one hipGraph and replayed (how the engines run
    them), so the figure is the device cost, not the host's per-call Python / launch overhead (~3 us
    per eager call here, more than the W=1 kernels themselves).  Falls back to eager launches when a
    route cannot be captured.  Every rank replays the same number of times."""
    torch.cuda.synchronize(device)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g = None
    if os.environ.get("PDE_ROUTE_TIMING", "graph") == "graph":
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(iters):
                    fn()
        except Exception:   # pragma: no cover - capture not supported for this route
            g = None
            torch.cuda.synchronize(device)
        if group is not None and group.size() > 1:   # every rank replays, or none does
            if _host_allreduce_max_f64(group, [0.0 if g is not None else 1.0])[0] > 0:
                g = None
    if g is not None:
        g.replay()                                   # warm replay
        s.record()
        for _ in range(3):
            g.replay()
        e.record()
        torch.cuda.synchronize(device)
        return s.elapsed_time(e) * 1e3 / (3 * iters)   # us per call
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize(device)
    return s.elapsed_time(e) * 1e3 / iters   # us per call


def tune_routes(group, peer: Optional[PeerAllReduce], rccl_fn, sizes: Iterable[int], device,
                dtype=torch.float32, iters: int = 30, bufs: Optional[dict] = None):
    """Fastest all-reduce route per element count: ({numel: 'rccl' | 'peer1' | 'peer2'},
    {numel: {candidate: us per call (max over ranks)}}).

    ``rccl_fn(tensor)`` enqueues the RCCL all-reduce on the current stream (None: RCCL unavailable).
    Every candidate is timed on every rank; the per-candidate MAX over ranks decides, so all ranks
    agree.  Forced with PDE_ALLREDUCE_ROUTE=rccl|peer1|peer2."""
    forced = os.environ.get("PDE_ALLREDUCE_ROUTE")
    out: Dict[int, str] = {}
    timings: Dict[int, dict] = {}
    for n in sizes:
        cands = []
        if rccl_fn is not None:
            cands.append(RCCL)
        buf = None
        if peer is not None and peer.ok:
            # the tensor the route will run on (a registered buffer times the in-place kernel)
            buf = bufs[n] if bufs and n in bufs else torch.zeros(n, device=device, dtype=dtype)
            if peer.supports(buf):
                cands += [ONE_SHOT, TWO_SHOT]
        if forced in cands:
            out[n] = forced
            continue
        if not cands:
            raise RuntimeError("no all-reduce route available")
        if len(cands) == 1:
            out[n] = cands[0]
            continue
        times = []
        if buf is None:
            buf = bufs[n] if bufs and n in bufs else torch.zeros(n, device=device, dtype=dtype)
        for c in cands:
            fn = (lambda: rccl_fn(buf)) if c == RCCL else (lambda c=c: peer.all_reduce_(buf, c))
            fn()
            group.host.barrier()
            times.append(_time_calls(fn, iters, device, group))
        times = _host_allreduce_max_f64(group, times)
        out[n] = cands[min(range(len(cands)), key=lambda i: times[i])]
        timings[n] = dict(zip(cands, [round(t, 2) for t in times]))
    return out, timings
