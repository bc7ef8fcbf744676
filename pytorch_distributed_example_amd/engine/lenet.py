"""Fused, graph-capturable data-parallel training step for the reference toy CNN.

Per step (reference semantics: /root/reference/mnist/main.py:84-99 forward, cross_entropy,
zero_grad, backward, average_gradients, Adam step, meters) this issues:

  compute stream : F1 conv1+conv2 (+gather, +grad zeroing) -> F2 fc1 -> F3 head/loss/dlogits
                   -> B1 fc backward --(event)--> B2 conv backward --(event)--> [wait comm] -> fused Adam
  comm stream    :                    all_reduce(bucket 0: fc grads, 1.62 MB) | all_reduce(bucket 1: conv grads)

(the "overlap" schedule; W > 1 picks overlap / flat / serial and a route per bucket -- RCCL or the
xGMI peer kernel -- by timing whole steps on the node: ``autotune_schedule``)

* Gradients live in one flat buffer laid out in bucket order (``parallel.flat``); bucket 0 (fc1/fc2,
  94 % of the bytes) is complete after B1, so its all-reduce overlaps the conv backward (B2).
* The 1/world_size average of ``average_gradients`` (main.py:122-127) is folded into Adam's
  ``grad_scale``; all-reduces are plain SUMs on the flat bucket views.
* Loss/accuracy meters accumulate on the device and are read once per epoch (no per-step
  ``.item()`` syncs, survey S1).
* The dataset is device resident; the epoch permutation is uploaded once per epoch and batch b of
  the epoch is gathered inside F1 from a device batch counter that F2 advances, so a
  captured hipGraph replays consecutive steps with no host work at all.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from .._ext import kernels
from ..ops.lenet_fused import pack_conv2_weight
from ..parallel.flat import FlatLayout

FC_BUCKET = ["fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"]
CONV_BUCKET = ["conv1.weight", "conv1.bias", "conv1.grad_replicas", "conv2.weight", "conv2.bias"]   # v1
CONV_BUCKET_V2 = ["conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias"]
C1_NREP = 16          # conv1 gradient replicas (atomic contention: 128 images -> 8 adders per address)
C1_STRIDE = 576       # conv1.weight (500 -> 512 slot) + conv1.bias (20 -> 64 slot); v2: int64 [500 | 20] + pad
C2_NREP = 16          # conv2 wgrad slabs of the v2 step (one per 8-image group, folded inside the launch)
C2_STRIDE = 25088     # slab: conv2.weight [25000] | pad | conv2.bias [50] at 25024


class LeNetTrainStep:
    def __init__(self, net: torch.nn.Module, batch_size: int = 128, lr: float = 1e-3, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, optimizer: str = "adam", momentum: float = 0.0,
                 comm=None, overlap: bool = True, force_comm: bool = False, v2: Optional[bool] = None):
        self.net = net
        p0 = next(net.parameters())
        if not p0.is_cuda:
            raise ValueError("LeNetTrainStep needs the model on a GPU")
        self.device = p0.device
        self.B = int(batch_size)
        self.lr, self.betas, self.eps, self.wd = float(lr), tuple(betas), float(eps), float(weight_decay)
        self.optimizer = optimizer
        self.momentum = float(momentum)
        self.comm = comm
        self.world = comm.world_size if comm is not None else 1
        # communication schedule (W > 1): "overlap" = fc bucket all-reduced on the comm stream beside
        # the conv backward (conv bucket on the comm stream too: four cross-stream edges per step);
        # "overlap2" = the same fc overlap, the conv bucket after it on the comm stream and one join
        # before the whole optimizer (three edges); "flat" = one all-reduce on the comm stream after backward; "serial" = one
        # all-reduce on the compute stream (no cross-stream edges: in a hipGraph each edge between
        # kernels on different streams measured 5-9 us, see autotune_schedule); "fused" = the fc
        # bucket is all-reduced by side blocks of the conv backward kernel (xGMI peer protocol), the
        # conv bucket after it on the compute stream
        self.mode = "overlap" if overlap else "flat"
        self._peer_dev = None
        self._ipdev = None            # PeerIpDev bytes of the registered flat gradients ("pfold" route)
        self._fold_sync = None
        self.ar_epoch = torch.full((1,), -1, device=p0.device, dtype=torch.int64)   # fused-Adam all-reduce
        # force_comm: run the comm-stream/event path even at world size 1 (1-GPU testing of the W>1 path)
        self.comm_on = comm is not None and (self.world > 1 or force_comm)
        self.K = kernels()
        dev = self.device
        # v2 step (csrc/kernels/lenet_v2.hip): prefetched batches, LDS-DMA weight staging, 8-wave conv
        # forward, co-resident conv backward that reduces its weight gradients deterministically inside
        # the launch (conv2: 16 per-image-group slabs folded in group order by the last-arriving block
        # of each k slice; conv1: order-free int64 fixed-point sums) into the canonical gradient slots,
        # so the all-reduced conv bucket is exactly the conv parameters.  At W = 1 with Adam the same
        # launch also runs the optimizer (no separate Adam kernel: the folding blocks update the conv
        # parameters, every W block one float4 of the fc parameters).  v1 (lenet.hip) for B > 128.
        self.v2 = ((os.environ.get("PDE_LENET_V2", "1") != "0") if v2 is None else bool(v2)) and self.B <= 128
        # where the conv weight gradients are reduced (v2):
        #   "defer" (W = 1): the conv backward leaves 16 conv2 slabs (plain stores) and 16 conv1 replicas
        #           (float atomics) in the flat buffer; the optimizer's fold blocks sum them in fixed order
        #           -- no reduction seam on the chain (measured: an in-launch fold + Adam is 2-3 us slower);
        #   "ext"   (comm path default): the conv backward stores 16 conv2 slabs and one conv1 partial per
        #           image with plain stores (no atomics, no arrival tickets), and a small fold launch
        #           (k_conv_grad_fold) sums them in fixed order into the canonical slots, so the
        #           all-reduced conv bucket is exactly the conv parameters and bit-reproducible
        #           (round 3's in-launch "fold" cost 4.4 us on the chain: profiles/r3_lenet/phases_fold.txt);
        #   "fold"  the in-launch reduction (last-arriving W block per k slice; conv1 as int64 fixed-point
        #           sums): used by the "fused" schedules, whose peer side blocks live in that kernel.
        # PDE_LENET_BWD_MODE=fold|ext forces a comm-path reduction at W = 1 (A/B runs, tests).
        mode = os.environ.get("PDE_LENET_BWD_MODE", "defer")
        if mode not in ("defer", "fold", "ext"):
            raise ValueError(f"PDE_LENET_BWD_MODE must be 'defer', 'fold' or 'ext', not {mode!r}")
        if self.comm_on and mode == "defer":
            mode = "ext"
        self.bwd_mode = mode if self.v2 else "v1"
        dev = self.device
        named = [(n, tuple(p.shape)) for n, p in net.named_parameters()]
        if self.bwd_mode == "defer":
            # gradient replicas in the flat buffer (replica 0 = the canonical slot), folded in fixed order
            # by the optimizer's fold blocks: conv1 as 16 atomic-add replicas, conv2 as 16 image-group slabs
            self.layout = FlatLayout(named, [FC_BUCKET, CONV_BUCKET + ["conv2.grad_replicas"]],
                                     extra_shapes={"conv1.grad_replicas": ((C1_NREP - 1) * C1_STRIDE,),
                                                   "conv2.grad_replicas": ((C2_NREP - 1) * C2_STRIDE,)})
        elif self.v2:
            self.layout = FlatLayout(named, [FC_BUCKET, CONV_BUCKET_V2])
        else:
            self.layout = FlatLayout(named, [FC_BUCKET, CONV_BUCKET],
                                     extra_shapes={"conv1.grad_replicas": ((C1_NREP - 1) * C1_STRIDE,)})
        self.params, self.grads = self.layout.bind(net)
        V = self.layout.view
        self.p = {n: V(self.params, n) for n in self.layout.param_names}
        self.g = {n: V(self.grads, n) for n in self.layout.param_names}
        self.off = {n: self.layout.slots[n].offset for n in self.layout.param_names}
        c1 = self.off["conv1.weight"]
        self.c1_off = c1
        self.c2_off = self.off["conv2.weight"]
        self.bucket_grads = [self.layout.bucket_view(self.grads, i) for i in range(2)]
        o = self.off
        assert o["conv1.bias"] == c1 + 512 and o["conv2.bias"] == self.c2_off + 25024
        if self.v2:
            self.c1rep = torch.zeros(C1_NREP * C1_STRIDE, device=dev, dtype=torch.int64)   # kept zero by the kernel
            self.tick = torch.zeros(32, device=dev, dtype=torch.int32)                      # arrival counters
        if self.bwd_mode == "defer":
            assert self.layout.slots["conv1.grad_replicas"].offset == c1 + C1_STRIDE
            assert self.layout.slots["conv2.grad_replicas"].offset == self.c2_off + C2_STRIDE
            self.c1part = self.grads[c1: c1 + C1_NREP * C1_STRIDE]
            self.slab = self.grads[self.c2_off: self.c2_off + C2_NREP * C2_STRIDE]
            self.zero_view = self.c1part              # zeroed by the conv forward (atomic targets)
        elif self.v2:
            assert o["conv2.weight"] == c1 + C1_STRIDE
            self.slab = torch.zeros(C2_NREP * C2_STRIDE, device=dev, dtype=torch.float32)
            self.c1part = torch.zeros(C1_NREP * C1_STRIDE, device=dev, dtype=torch.float32)   # unused in fold mode
            self.c1img = torch.zeros(self.B * 520, device=dev, dtype=torch.float32)          # ext mode
            self.zero_view = None
        else:
            assert self.layout.slots["conv1.grad_replicas"].offset == c1 + C1_STRIDE
            self.g_c1w_rep = self.grads[c1: c1 + C1_NREP * C1_STRIDE]
            self.g_c1b_rep = self.grads[c1 + 512: c1 + C1_NREP * C1_STRIDE]
            self.zero_view = self.bucket_grads[1]
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params) if optimizer == "adam" else self.m
        self.counters = torch.zeros(2, device=dev, dtype=torch.int64)   # [optimizer step, batch in epoch]
        self.arrive = torch.zeros(1, device=dev, dtype=torch.int32)
        if self.v2:
            self.Wp = torch.zeros(2 * 72 * 256, device=dev, dtype=torch.float32)   # padding stays zero
            self.K.lenet_pack_w2_v2(self.p["conv2.weight"].detach().contiguous(), self.Wp)
            self.Wt2 = None
        else:
            self.Wt2 = pack_conv2_weight(self.p["conv2.weight"])
        self.pack_off = self.layout.slots["conv2.weight"].offset
        f32 = dict(device=dev, dtype=torch.float32)
        B = self.B
        self.P1 = torch.empty(B * 2880, **f32)
        self.A1 = torch.empty(B * 2880, device=dev, dtype=torch.uint8)
        self.P2 = torch.empty(B * 800, **f32)
        self.A2 = torch.empty(B * 800, device=dev, dtype=torch.uint8)
        self.H1 = torch.empty(B * 500, **f32)
        self.dZ1 = torch.empty(B * 500, **f32)
        self.dZ2 = torch.empty(B * 10, **f32)
        self.dP2m = torch.empty(B * 800, **f32)
        self.cur_row = torch.zeros(B, device=dev, dtype=torch.int32)
        self.cur_lbl = torch.zeros(B, device=dev, dtype=torch.int64)
        # v2 prefetch buffers, double-buffered by step parity q (host-tracked; baked into captured graphs)
        self.Xb = torch.zeros(2, B, 784, **f32)
        self.Yb = torch.zeros(2, B, device=dev, dtype=torch.int64)
        self.rowsb = torch.zeros(2, B, device=dev, dtype=torch.int32)
        self.q = 0
        self.row_loss = torch.zeros(B, **f32)
        self.row_hit = torch.zeros(B, device=dev, dtype=torch.int32)
        self.loss_sum = torch.zeros(1, device=dev, dtype=torch.float64)
        self.correct = torch.zeros(1, device=dev, dtype=torch.int64)
        self.samples = 0
        self.eval_loss = torch.zeros(1, device=dev, dtype=torch.float64)
        self.eval_correct = torch.zeros(1, device=dev, dtype=torch.int64)
        self.comm_stream = torch.cuda.Stream(device=dev) if self.comm_on else None
        self._ev = {k: torch.cuda.Event() for k in ("fc", "conv", "fc_done")}
        self.bucket_ranges = [tuple(r) for r in self.layout.bucket_ranges]
        assert self.bucket_ranges[0][0] == 0 and self.bucket_ranges[1][0] >= self.bucket_ranges[0][1]
        if self.comm_on and hasattr(comm, "enable_peer") and not comm.routes:
            # small buckets: time the xGMI peer all-reduce against RCCL at exactly these sizes, on the
            # flat gradient buffer itself, registered so the peer routes read it in place
            bufs = {b.numel(): b for b in self.bucket_grads}
            bufs[self.grads.numel()] = self.grads
            comm.enable_peer(list(bufs), dev, inplace=self.grads, bufs=bufs)
        self.X = self.Y = self.idx = None
        self.nbatches = 0
        self.graphs = {}
        self.bwd_dbg = 0          # ablation switch of the v2 conv backward (tools/lenet_phases.py only)

    # ------------------------------------------------------------------ data binding
    def bind_dataset(self, images: torch.Tensor, labels: torch.Tensor):
        if images.device != self.device or labels.device != self.device:
            raise ValueError("dataset must be resident on the training device")
        self.X = images.reshape(images.shape[0], 784).contiguous()
        self.Y = labels.to(torch.int64).contiguous()

    def set_epoch_indices(self, idx: torch.Tensor):
        """Upload this epoch's (rank-local) sample order; batches are [i*B, (i+1)*B) plus a ragged tail."""
        idx = idx.to(self.device, torch.int32).contiguous()
        n = idx.numel()
        if self.idx is not None and self.idx.numel() == n:
            self.idx.copy_(idx)          # keep the address captured by existing graphs
        else:
            self.idx = idx
            self.graphs.clear()
        self.nfull = n // self.B
        self.tail = n - self.nfull * self.B
        self.nbatches = self.nfull + (1 if self.tail else 0)
        self.counters[1].zero_()
        if self.v2:      # prefetch batch 0 of the epoch into the current parity's buffers
            self.K.lenet_gather(self.X, self.Y, self.idx, None, self.nbatches, self.B, self.Xb[self.q],
                                self.Yb[self.q], self.rowsb[self.q])

    # ------------------------------------------------------------------ the step
    def _opt(self, lo: int, hi: int, conv: bool, fuse_ar: Optional[str] = None):
        """Fused optimizer update of the flat range [lo, hi) (one bucket or everything).  The conv
        range carries the conv2 weight repack (Wp / Wt2) and, in the v1 layout, the conv1
        gradient-replica fold (v2 writes canonical gradients, nothing to fold).
        ``fuse_ar`` ('adam1' / 'adam2'): side blocks of the Adam kernel all-reduce the conv bucket
        (one- / two-shot peer protocol) while the other blocks update the fc parameters."""
        K, sl = self.K, slice(lo, hi)
        pack_off = self.pack_off - lo if conv else -1
        pack, mode = (self.Wp, 2) if self.v2 else (self.Wt2, 1)
        if not conv:
            pack = None
        folds = {}
        if conv and self.bwd_mode == "v1":        # in-layout float conv1 replicas
            folds = dict(fold_off=self.c1_off - lo, fold_len=C1_STRIDE, fold_nrep=C1_NREP, fold_stride=C1_STRIDE)
        elif conv and self.bwd_mode == "defer":   # conv2 slabs + int64 conv1 replicas of the conv backward
            folds = dict(fold_off=self.c1_off - lo, fold_len=C1_STRIDE, fold_nrep=C1_NREP, fold_stride=C1_STRIDE,
                         fold2_off=self.c2_off - lo, fold2_len=C2_STRIDE, fold2_nrep=C2_NREP, fold2_stride=C2_STRIDE)
        scale = 1.0 / self.world
        if self.optimizer == "adam":
            far = {}
            if fuse_ar is not None:
                far = dict(peer_dev=self._peer_device_args(), ar_off=self.bucket_ranges[1][0] - lo,
                           ar_epoch=self.ar_epoch, ar_two=int(fuse_ar == "adam2"))
            K.adam_flat(self.params[sl], self.grads[sl], self.m[sl], self.v[sl], self.lr, self.betas[0],
                        self.betas[1], self.eps, self.wd, False, scale, self.counters, self.arrive, -1, pack_off,
                        pack, pack_mode=mode, **folds, **far)
        else:
            K.sgd_flat(self.params[sl], self.grads[sl], self.m[sl], self.lr, self.momentum, 0.0, self.wd, False,
                       scale, self.counters, self.arrive, -1, pack_off, pack, pack_mode=mode, **folds)

    def _fold_ar(self, B: int, two: bool = False):
        """The "serial ...:pfold" / "pfold2" routes: the ext-mode conv-gradient fold and the in-place
        one-shot / two-shot all-reduce of the whole flat gradient buffer in ONE launch
        (k_conv_fold_ar / k_conv_fold_ar2, lenet_v2.hip)."""
        if self._ipdev is None:
            peer = self.comm.peer
            rid, off = peer.registered_range(self.grads)
            assert off == 0
            self._ipdev = torch.frombuffer(bytearray(peer.native.registered_device_args(rid)), dtype=torch.uint8)
            self._fold_sync = torch.zeros(2, device=self.device, dtype=torch.int32)
        o = self.off
        lo, hi = self.bucket_ranges[1]
        self.K.lenet_conv_fold_ar(self._ipdev, self.slab, self.c1img, B, self.grads, o["conv1.weight"],
                                  o["conv1.bias"], o["conv2.weight"], o["conv2.bias"], lo, hi, self._fold_sync, 1.0,
                                  int(two))

    def pfold_ok(self, two: bool = False) -> bool:
        """The fused fold + all-reduce route is available: v2 ext-mode layout, the flat gradient buffer
        registered for the in-place peer route, and (one-shot) one grid that fits the peer grid cap."""
        peer = getattr(self.comm, "peer", None) if self.comm is not None else None
        if not self.v2 or self.bwd_mode != "ext" or peer is None or peer.native is None:
            return False
        reg = peer.registered_range(self.grads)
        if reg is None or reg[1] != 0 or self.grads.numel() % 4:
            return False
        if two:
            return True
        n4 = self.grads.numel() // 4
        return (n4 + 2047) // 2048 <= min(256, 256 // max(1, getattr(peer, "shared", 1)))

    def _conv_bwd2(self, B: int, q: int, fused_fc_route: Optional[str] = None, fold: bool = True):
        """The v2 conv backward (+ the next batch's prefetch and the meters); ``fused_fc_route``
        ('peer1' / 'peer2'): its W blocks also all-reduce the fc bucket across ranks once their own work
        is done."""
        p = self.p
        kw = dict(row_loss=self.row_loss, row_hit=self.row_hit, loss_sum=self.loss_sum, correct=self.correct,
                  gX=self.X, glabels=self.Y, gidx=self.idx, gctr=self.counters[1:], gnbatches=self.nbatches,
                  gstride=self.B, gXdst=self.Xb[1 - q], gYdst=self.Yb[1 - q], grows=self.rowsb[1 - q],
                  dbg=self.bwd_dbg)
        if fused_fc_route is not None:
            kw.update(peer_dev=self._peer_device_args(), ar_buf=self.bucket_grads[0],
                      ar_two=int(fused_fc_route == "peer2"))
        # the fused schedules' peer side blocks live in the in-launch "fold" kernel variant
        mode = "fold" if fused_fc_route is not None else self.bwd_mode
        kw["defer"] = {"fold": 0, "defer": 1, "ext": 2}[mode]
        if mode == "ext":
            kw["c1img"] = self.c1img
        o = self.off
        self.K.lenet_conv_bwd2(self.Xb[q], self.P1, self.A1, self.dP2m, self.A2, p["conv2.weight"], B, self.slab,
                               self.c1rep, self.c1part, self.tick, self.grads, o["conv1.weight"], o["conv1.bias"],
                               o["conv2.weight"], o["conv2.bias"], **kw)
        if mode == "ext" and fold:   # canonical conv gradients (fixed-order sums) for the conv-bucket all-reduce
            self.K.lenet_conv_grad_fold(self.slab, self.c1img, B, self.grads, o["conv1.weight"], o["conv1.bias"],
                                        o["conv2.weight"], o["conv2.bias"])

    def _launch(self, B: int):
        """One step on the current stream: conv_fwd -> fc1 -> head -> fc_bwd -> conv_bwd -> opt.

        With a comm group and ``overlap``, bucket 0 (fc grads, complete after fc_bwd) is all-reduced
        on the comm stream while conv_bwd runs; bucket 1 after conv_bwd; the optimizer waits for both.

        (Measured and rejected: moving the fc weight-gradient roles and the fc-bucket optimizer to a
        side stream beside conv_bwd -- conv_bwd already fills the GPU, so it slowed from 24 to 31 us,
        and the two cross-stream joins cost 5-7 us each: 91 us/step vs 81 us single-stream.  Also
        rejected: folding the head into fc1, the last column block of each 16-row tile running the
        head -- with __threadfence() in every block (L2 write-back/invalidate per block) 99 us/step,
        with write-through H1 stores + agent-scope loads 83 us, against 69 us for two launches: one
        wave doing 4 latency-bound rows serially costs more than the kernel boundary it saves.  Round 2:
        the head without its launch -- fc1 blocks atomically accumulating H1 W2^T into a logits buffer,
        every fc_bwd block finishing log_softmax / CE / dz and building its dZ1 / dZ2 operand in LDS --
        measured 74.3 us/step against 57.7: fc1 + 2 us (cross-XCD float atomics drain 8.8 us before the
        next launch), fc_bwd 5.8 -> 19 us (per-block head + operand build, and 37 KB of LDS halving the
        resident blocks); profiles/r2_lenet_v3/rejected_fused_head/.  Also rejected in round 2: the fc
        parameters' Adam as extra blocks of the conv backward launch -- they dispatch only as W blocks
        retire and end after the D chain (conv_bwd 18.5 -> 21.4 us), while the remaining conv-range
        Adam is latency-bound on the slab folds (6.3 -> 5.6 us): 61.1 vs 57.7 us/step;
        profiles/r2_lenet_v3/rejected_fc_adam_in_bwd/.  A persistent single-launch step was not built: a
        grid-wide barrier (one agent-scope atomic counter, co-resident blocks) measures 3.6 us at 128
        blocks and 10.4 us at 256 against 1.5-1.6 us for a kernel boundary in a stream or hipGraph
        (tools/native/grid_barrier_bench.hip, profiles/r2_lenet_v3/grid_barrier_vs_kernel_boundary.jsonl).)"""
        K, p, g = self.K, self.p, self.g
        q = self.q
        if self.v2:
            K.lenet_conv_fwd2(self.Xb[q], B, p["conv1.weight"], p["conv1.bias"], self.Wp, p["conv2.bias"], self.P1,
                              self.A1, self.P2, self.A2, self.zero_view)
            rows, labels = self.rowsb[q], self.Yb[q]
        else:
            K.lenet_conv_fwd(self.X, self.idx, self.counters[1:], self.nbatches, self.B, self.Y, B,
                             p["conv1.weight"], p["conv1.bias"], self.Wt2, p["conv2.bias"], self.P1, self.A1, self.P2,
                             self.A2, self.cur_row, self.cur_lbl, self.bucket_grads[1])
            rows, labels = self.cur_row, self.cur_lbl
        K.lenet_fc1_fwd(self.P2, B, p["fc1.weight"], p["fc1.bias"], self.H1, self.counters)   # bumps counters
        K.lenet_head(self.H1, B, p["fc2.weight"], p["fc2.bias"], labels, 1.0 / B, None, self.dZ2, self.dZ1,
                     self.row_loss, self.row_hit, None, None)
        if self.v2:
            self.q = 1 - q
        fused = self.comm_on and self.mode == "fused"
        # the loss / accuracy meters are folded by an extra block of conv_bwd (off fc_bwd's chain)
        fc_args = (self.P2, self.H1, self.dZ1, self.dZ2, p["fc1.weight"], B, self.dP2m, g["fc1.weight"],
                   g["fc1.bias"], g["fc2.weight"], g["fc2.bias"], None, None, None, None)
        cur = torch.cuda.current_stream(self.device)
        ev, cs = self._ev, self.comm_stream
        K.lenet_fc_bwd(*fc_args)
        pfold = (self.comm.routes.get(self.grads.numel()) if self.comm_on and self.mode == "serial" else None)
        pfold = pfold if pfold in ("pfold", "pfold2") else None
        if self.v2:
            conv_bwd = lambda: self._conv_bwd2(B, q, fold=not pfold)
        else:
            conv_args = (self.X, rows, self.P1, self.A1, self.dP2m, self.A2, p["conv2.weight"], B,
                         self.g_c1w_rep, self.g_c1b_rep, g["conv2.weight"], g["conv2.bias"], C1_NREP, C1_STRIDE,
                         self.row_loss, self.row_hit, self.loss_sum, self.correct)
            conv_bwd = lambda: K.lenet_conv_bwd(*conv_args)
        if fused:
            fc_route = self.comm.routes.get(self.bucket_grads[0].numel(), "peer2")
            if self.v2:
                self._conv_bwd2(B, q, fused_fc_route=fc_route)
            else:
                K.lenet_conv_bwd(*conv_args, 0, self._peer_device_args(), self.bucket_grads[0],
                                 int(fc_route == "peer2"))
            conv_route = self.comm.routes.get(self.bucket_grads[1].numel(), "rccl")
            if conv_route in ("adam1", "adam2") and self.optimizer == "adam":
                self._opt(0, self.params.numel(), True, fuse_ar=conv_route)
            else:
                self.comm.all_reduce_(self.bucket_grads[1])
                self._opt(0, self.params.numel(), True)
            return
        if self.comm_on and self.mode in ("overlap", "overlap2"):
            ev["fc"].record(cur)
            cs.wait_event(ev["fc"])
            with torch.cuda.stream(cs):
                self.comm.all_reduce_(self.bucket_grads[0])
        conv_bwd()
        if self.comm_on and self.mode == "overlap2":
            # three cross-stream edges per step instead of four: both buckets are reduced on the comm
            # stream (one communicator, one stream: collectives stay ordered), then ONE join before the
            # whole optimizer (no separate fc-range update beside the conv bucket's reduction)
            ev["conv"].record(cur)
            cs.wait_event(ev["conv"])
            with torch.cuda.stream(cs):
                self.comm.all_reduce_(self.bucket_grads[1])
            cur.wait_stream(cs)
            self._opt(0, self.params.numel(), True)
            return
        if not self.comm_on or self.mode == "none":     # "none": the comm path's compute alone (autotune probe)
            self._opt(0, self.params.numel(), True)
            return
        if self.mode == "serial":
            if pfold:
                self._fold_ar(B, two=pfold == "pfold2")   # fold + all-reduce in one launch
            else:
                self.comm.all_reduce_(self.grads)
            self._opt(0, self.params.numel(), True)
            return
        ev["conv"].record(cur)
        cs.wait_event(ev["conv"])
        if self.mode == "flat":
            with torch.cuda.stream(cs):
                self.comm.all_reduce_(self.grads)
            cur.wait_stream(cs)
            self._opt(0, self.params.numel(), True)
            return
        # the fc-bucket update (94 % of the parameters) runs while the conv bucket is being reduced
        ev["fc_done"].record(cs)
        with torch.cuda.stream(cs):
            self.comm.all_reduce_(self.bucket_grads[1])
        (a0, a1), (b0, b1) = self.bucket_ranges
        cur.wait_event(ev["fc_done"])
        self._opt(a0, a1, False)
        cur.wait_stream(cs)
        self._opt(b0, b1, True)

    def _peer_device_args(self):
        if self._peer_dev is None:
            peer = getattr(self.comm, "peer", None)
            if peer is None or peer.native is None:
                raise RuntimeError("the fused schedule needs the xGMI peer all-reduce")
            self._peer_dev = torch.frombuffer(bytearray(peer.native.device_args()), dtype=torch.uint8)
        return self._peer_dev

    @property
    def overlap(self) -> bool:
        return self.mode == "overlap"

    def _batch_size_at(self, b: int) -> int:
        return self.B if b < self.nfull else self.tail

    def step(self, B: Optional[int] = None):
        """Run one training step eagerly (B defaults to the full batch size)."""
        self._launch(B or self.B)

    def capture(self, B: Optional[int] = None, warmup: int = 0, steps: int = 1):
        """Capture ``steps`` consecutive steps of batch size B into one hipGraph (replayed by
        ``replay``).  Every step reads its batch position / optimizer step from device counters, so
        a multi-step graph is just the step chain repeated; it amortises the per-replay launch cost.
        The v2 step alternates its prefetch buffers by step parity: a graph is keyed by the parity it
        starts at (capturing does not execute, so the host parity is restored afterwards)."""
        B = B or self.B
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._launch(B)
        torch.cuda.current_stream(self.device).wait_stream(s)
        q0 = self.q
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(steps):
                self._launch(B)
        self.q = q0
        self.graphs[(B, steps, q0)] = g
        return g

    def prime_graphs(self, step_counts=(1,), B: Optional[int] = None, replays: int = 1):
        """Capture the graphs of every step count at BOTH step parities (v2 prefetch buffers) and
        launch each ``replays`` times (untimed first launches), leaving the parity as it was."""
        B = B or self.B
        q0 = self.q
        parities = (0, 1) if self.v2 else (q0,)
        for S in step_counts:
            for par in parities:
                self.q = par
                if (B, S, par) not in self.graphs:
                    self.capture(B, steps=S)
        self.q = q0
        if self.v2 and (B, 1, 0) not in self.graphs:
            for par in (0, 1):
                self.q = par
                self.capture(B, steps=1)
            self.q = q0
        for _ in range(replays):
            for S in step_counts:
                if not self.v2:
                    self.replay(B, steps=S)
                elif S % 2:                           # odd: two replays visit both parities
                    self.replay(B, steps=S)
                    self.replay(B, steps=S)
                else:                                 # even: a 1-step replay moves to the other parity
                    self.replay(B, steps=S)
                    self.replay(B, steps=1)
                    self.replay(B, steps=S)
                    self.replay(B, steps=1)

    def replay(self, B: Optional[int] = None, steps: int = 1):
        """Run ``steps`` steps through the (captured on first use) graph of that many steps."""
        B = B or self.B
        g = self.graphs.get((B, steps, self.q))
        if g is None:
            g = self.capture(B, steps=steps)
            # capturing does not execute: replay now so call semantics stay "steps steps"
        g.replay()
        if self.v2 and steps % 2:
            self.q = 1 - self.q

    # ------------------------------------------------------------------ epochs / meters
    def run_epoch(self, use_graph: bool = True):
        """All batches of the bound epoch (full batches via graph replay, then the ragged tail)."""
        for b in range(self.nbatches):
            Bb = self._batch_size_at(b)
            if use_graph:
                self.replay(Bb)
            else:
                self.step(Bb)
        self.samples += self.nfull * self.B + self.tail

    def reset_meters(self):
        """Zero the device meters without a host round trip (enqueued on the current stream)."""
        self.loss_sum.zero_()
        self.correct.zero_()
        self.samples = 0

    def read_meters(self, reset: bool = True):
        loss = float(self.loss_sum.item())
        correct = int(self.correct.item())
        n = self.samples
        if reset:
            self.loss_sum.zero_()
            self.correct.zero_()
            self.samples = 0
        return loss, correct, n

    @torch.no_grad()
    def evaluate(self, images: torch.Tensor, labels: torch.Tensor, batch_size: Optional[int] = None):
        """Forward-only pass over a (device) test set with the fused kernels; returns (loss_sum, correct, n)."""
        K, p = self.K, self.p
        bs = batch_size or self.B
        X = images.reshape(images.shape[0], 784).contiguous()
        Y = labels.to(torch.int64).contiguous()
        n = X.shape[0]
        self.eval_loss.zero_()
        self.eval_correct.zero_()
        P1 = torch.empty(bs * 2880, device=self.device)
        A1 = torch.empty(bs * 2880, device=self.device, dtype=torch.uint8)
        P2 = torch.empty(bs * 800, device=self.device)
        A2 = torch.empty(bs * 800, device=self.device, dtype=torch.uint8)
        H1 = torch.empty(bs * 500, device=self.device)
        for s in range(0, n, bs):
            B = min(bs, n - s)
            if self.v2:
                K.lenet_conv_fwd2(X[s:s + B], B, p["conv1.weight"], p["conv1.bias"], self.Wp, p["conv2.bias"], P1,
                                  A1, P2, A2)
            else:
                K.lenet_conv_fwd(X[s:s + B], None, None, 0, 0, None, B, p["conv1.weight"], p["conv1.bias"],
                                 self.Wt2, p["conv2.bias"], P1, A1, P2, A2, None, None, None)
            K.lenet_fc1_fwd(P2, B, p["fc1.weight"], p["fc1.bias"], H1, None)
            K.lenet_head(H1, B, p["fc2.weight"], p["fc2.bias"], Y[s:s + B], 1.0 / B, None, None, None,
                         None, None, self.eval_loss, self.eval_correct)
        return float(self.eval_loss.item()), int(self.eval_correct.item()), n

    # ------------------------------------------------------------------ optimizer state (torch format)
    def optimizer_state_dict(self):
        """``torch.optim.Adam.state_dict()``-compatible dict (params indexed in registration order)."""
        names = list(self.layout.param_names)
        step = float(self.counters[0].item())
        state = {}
        for i, n in enumerate(names):
            st = {"step": torch.tensor(step)}
            if self.optimizer == "adam":
                st["exp_avg"] = self.layout.view(self.m, n).detach().clone()
                st["exp_avg_sq"] = self.layout.view(self.v, n).detach().clone()
            elif self.momentum:
                st["momentum_buffer"] = self.layout.view(self.m, n).detach().clone()
            state[i] = st
        group = {"lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.wd, "amsgrad": False,
                 "params": list(range(len(names)))} if self.optimizer == "adam" else {
            "lr": self.lr, "momentum": self.momentum, "weight_decay": self.wd, "dampening": 0.0,
            "nesterov": False, "params": list(range(len(names)))}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, sd):
        names = [n for n, _ in self.net.named_parameters()]
        for i, n in enumerate(names):
            st = sd["state"].get(i)
            if not st:
                continue
            if "exp_avg" in st:
                self.layout.view(self.m, n).copy_(st["exp_avg"])
                self.layout.view(self.v, n).copy_(st["exp_avg_sq"])
            if "momentum_buffer" in st and st["momentum_buffer"] is not None:
                self.layout.view(self.m, n).copy_(st["momentum_buffer"])
            self.counters[0].fill_(int(float(st["step"])))
        self.ar_epoch.fill_(-1)
        self.sync_params()

    def sync_params(self):
        """Re-derive kernel-side weight copies after parameters were changed externally."""
        if self.v2:
            self.K.lenet_pack_w2_v2(self.p["conv2.weight"].detach().contiguous(), self.Wp)
        else:
            pack_conv2_weight(self.p["conv2.weight"], self.Wt2)

    # ------------------------------------------------------------------ schedule autotuning (W > 1)
    def set_schedule(self, label: str):
        """Force one schedule by its autotuner label, e.g. ``"serial 431296:peer1"`` or
        ``"overlap2 25664:peer1,405632:rccl"`` (mode, then bucket numel:route pairs); identically on
        every rank (traces / A/B runs)."""
        mode, _, rest = label.strip().partition(" ")
        routes = {int(n): r for n, r in (kv.split(":") for kv in rest.split(",") if kv)}
        if mode not in ("overlap", "overlap2", "flat", "serial", "fused", "none"):
            raise ValueError(f"unknown schedule mode {mode!r}")
        self.mode = mode
        self.comm.routes = routes
        self.graphs.clear()

    def schedule_candidates(self):
        """(mode, {bucket numel: route}) pairs the comm path can run: bucketed + overlapped with the
        conv backward (one route per bucket), or one all-reduce after backward on the comm stream
        ("flat") or on the compute stream ("serial"), one route each."""
        routes = ["rccl"] if self.comm.group.rccl is not None else []
        if getattr(self.comm, "peer", None) is not None:
            routes += ["peer1", "peer2"]
        n0, n1, nall = (self.bucket_grads[0].numel(), self.bucket_grads[1].numel(), self.grads.numel())
        out = [("overlap", {n0: a, n1: b}) for a in routes for b in routes]
        out += [("overlap2", {n0: a, n1: b}) for a in routes for b in routes]
        out += [(m, {nall: a}) for m in ("flat", "serial") for a in routes]
        if getattr(self.comm, "peer", None) is not None:
            if self.pfold_ok():
                out += [("serial", {nall: "pfold"})]     # fold + in-place one-shot in one launch
            if self.pfold_ok(two=True) and self.world > 1:
                out += [("serial", {nall: "pfold2"})]    # fold + in-place two-shot in one launch
        if getattr(self.comm, "peer", None) is not None:
            out += [("fused", {n0: a, n1: b}) for a in ("peer1", "peer2") for b in routes]
            if self.optimizer == "adam":         # last: a failing candidate poisons the peer protocol
                out += [("fused", {n0: a, n1: b}) for a in ("peer1", "peer2") for b in ("adam1", "adam2")]
        # RCCL-only schedules first: they are timed even if the budget or the peer protocol runs out
        uses_peer = lambda c: c[0] == "fused" or any(r != "rccl" for r in c[1].values())
        return sorted(out, key=uses_peer)

    def autotune_schedule(self, steps: int = 40, graph_steps: int = 10, candidates=None,
                          budget_s: float = 60.0):
        """Pick the fastest communication schedule by timing WHOLE training steps on this node.

        Isolated all-reduce timings (``dist.peer.tune_routes``) miss the interaction with the kernels
        a collective overlaps (a peer kernel co-running with the conv backward competes for CUs, an
        RCCL kernel may not get a CU until it finishes), so every candidate schedule runs ``steps``
        real steps (hipGraph replays, as in training); the per-candidate MAX over ranks decides, so
        every rank picks the same one.  Model / optimizer / data-position state is snapshotted and
        restored: autotuning does not change training.  Returns {candidate label: us per step}.

        Bounded: candidates are timed in order (RCCL-only schedules first, the peer-protocol ones
        after) until ``budget_s`` of wall clock has passed; the stop decision is the MAX of the
        ranks' elapsed times, so every rank stops at the same candidate and the rest count as
        untimed.  A peer-protocol failure (barrier time-out) invalidates every later peer candidate
        on every rank; if no candidate survives, the RCCL-only "overlap" schedule is kept."""
        if not self.comm_on:
            return {}
        cands = candidates or self.schedule_candidates()
        state = [self.params, self.m, self.counters, self.Xb, self.Yb, self.rowsb] + (
            [self.v] if self.v is not self.m else [])
        snap = [t.clone() for t in state]
        q_saved = self.q
        saved_idx = None if self.idx is None else (self.idx, self.nfull, self.tail, self.nbatches)
        if self.idx is None or self.nfull < 1:
            raise RuntimeError("bind a dataset and set epoch indices before autotune_schedule")
        g = self.comm.group
        times, invalid = [], []
        peer = getattr(self.comm, "peer", None)
        wd = g.watchdog
        import time as _time
        t_start = _time.perf_counter()
        for mode, routes in cands:
            el = torch.tensor([_time.perf_counter() - t_start], dtype=torch.float64)
            g.host.allreduce(el.data_ptr(), 1, 1, 3)          # float64 MAX: one decision for all ranks
            if el.item() > budget_s:
                times.append(float("inf"))
                invalid.append(1)
                continue
            uses_peer = mode == "fused" or any(r != "rccl" for r in routes.values())
            perr0 = peer.error() if peer is not None else 0
            anyerr = torch.tensor([perr0], dtype=torch.int64)
            g.host.allreduce(anyerr.data_ptr(), 1, 3, 3)      # collective decision: every rank skips alike
            if uses_peer and anyerr.item():      # a timed-out peer protocol is poisoned: never pick it
                times.append(float("inf"))
                invalid.append(1)
                continue
            for t, s0 in zip(state, snap):       # every candidate starts from the same (replicated) state
                t.copy_(s0)
            self.q = q_saved
            self.ar_epoch.fill_(-1)              # optimizer steps repeat: no stale completion word
            self.sync_params()
            self.mode = mode
            self.comm.routes = dict(routes)
            self.graphs.clear()
            self.capture(steps=graph_steps)
            reps = max(1, steps // graph_steps)
            self.replay(steps=graph_steps)               # warm
            torch.cuda.synchronize(self.device)
            g.host.barrier()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                self.replay(steps=graph_steps)
            e.record()
            torch.cuda.synchronize(self.device)
            times.append(s.elapsed_time(e) * 1e3 / (reps * graph_steps))
            # safety net: a schedule must leave every replica bit-identical and report no comm error
            bits = self.params.view(torch.int32).to(torch.int64).sum().item()
            failed = (peer is not None and peer.error() > perr0) or (wd is not None and bool(wd.error()))
            invalid.append(1 if failed else 0)
            chk = torch.tensor([bits, -bits], dtype=torch.int64)
            g.host.allreduce(chk.data_ptr(), 2, 3, 3)          # int64 MAX: max(bits) and -min(bits)
            if chk[0].item() != -chk[1].item():
                invalid[-1] = 1
        # the same step with the collectives left out (never selectable): what the communication adds
        # on top of the comm path's compute (a W > 1 scaling point decomposes into the two)
        self.compute_only_us = None
        for tt, s0 in zip(state, snap):
            tt.copy_(s0)
        self.q = q_saved
        self.sync_params()
        self.mode = "none"
        self.graphs.clear()
        self.capture(steps=graph_steps)
        self.replay(steps=graph_steps)
        torch.cuda.synchronize(self.device)
        g.host.barrier()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = max(1, steps // graph_steps)
        s.record()
        for _ in range(reps):
            self.replay(steps=graph_steps)
        e.record()
        torch.cuda.synchronize(self.device)
        co = torch.tensor([s.elapsed_time(e) * 1e3 / (reps * graph_steps)], dtype=torch.float64)
        g.host.allreduce(co.data_ptr(), 1, 1, 3)
        self.compute_only_us = round(float(co.item()), 2)
        t = torch.tensor(times, dtype=torch.float64)
        g.host.allreduce(t.data_ptr(), t.numel(), 1, 3)     # float64 MAX over ranks
        bad = torch.tensor(invalid, dtype=torch.int64)
        g.host.allreduce(bad.data_ptr(), bad.numel(), 3, 3)  # int64 MAX: invalid anywhere -> invalid
        times = [float("inf") if b else x for x, b in zip(t.tolist(), bad.tolist())]
        if all(x == float("inf") for x in times):
            if g.rccl is None:
                raise RuntimeError("no communication schedule kept the replicas identical (comm failure?)")
            n0, n1 = self.bucket_grads[0].numel(), self.bucket_grads[1].numel()
            cands = list(cands) + [("overlap", {n0: "rccl", n1: "rccl"})]   # bounded fallback: RCCL only
            times.append(0.0)
        # a schedule with cross-stream edges (overlap / flat) must win by > 1 %: in a replayed hipGraph
        # every such edge adds 5-9 us of jitter-prone join latency (round 3: flat 61.9 us in the
        # autotuner, 68.3 us in the timed window; the single-stream serial schedule measured 62.0)
        eff = [x * (1.01 if cands[i][0] in ("overlap", "overlap2", "flat") else 1.0) for i, x in enumerate(times)]
        best = min(range(len(cands)), key=lambda i: eff[i])
        self.mode, self.comm.routes = cands[best][0], dict(cands[best][1])
        self.graphs.clear()
        # restore the training state the trial steps advanced
        for t, s0 in zip(state, snap):
            t.copy_(s0)
        self.q = q_saved
        self.ar_epoch.fill_(-1)
        self.sync_params()
        self.idx, self.nfull, self.tail, self.nbatches = saved_idx
        self.loss_sum.zero_()
        self.correct.zero_()
        torch.cuda.synchronize(self.device)
        label = lambda c: c[0] + " " + ",".join(f"{n}:{r}" for n, r in sorted(c[1].items()))
        self.schedule_times = {label(c): (round(x, 2) if x != float("inf") else None) for c, x in zip(cands, times)}
        self.schedule = label(cands[best])
        return self.schedule_times
