"""Reference-compatible training loop (``Average``, ``Accuracy``, ``Trainer``) plus the fused trainer.

``Trainer`` keeps the reference's API and printed format (/root/reference/mnist/main.py:15-127):
``Trainer(net, optimizer, train_loader, test_loader, device, distributed, do_eval).fit(epochs)``
with ``train()``, ``evaluate()`` and ``average_gradients()``.  Differences, all MI355X-motivated:
metrics accumulate on the device and are read once per epoch (the reference syncs twice per step
with ``.item()``), and the model's forward/backward runs the HIP kernels of ``ops``.

``FusedTrainer`` drives ``LeNetTrainStep`` (the whole step fused into 5 kernels + 1 Adam launch,
hipGraph-replayed) behind the same ``fit`` / print interface.
"""
from __future__ import annotations

import torch

from .. import dist, ops
from ..utils import profiling as prof


class Average(object):
    """Sample-weighted running mean (main.py:15-30)."""

    def __init__(self):
        self.sum = 0
        self.count = 0

    def update(self, value, number):
        self.sum += value * number
        self.count += number

    @property
    def average(self):
        return self.sum / self.count

    def __str__(self):
        return '{:.6f}'.format(self.average)


class Accuracy(object):
    """Top-1 accuracy (main.py:33-51); ``update`` keeps the count on the device (no per-step sync)."""

    def __init__(self):
        self.correct = 0
        self.count = 0

    def update(self, output, label):
        predictions = output.data.argmax(dim=1)
        correct = predictions.eq(label.data).sum()
        self.correct = self.correct + correct
        self.count += output.size(0)

    @property
    def accuracy(self):
        c = self.correct.item() if isinstance(self.correct, torch.Tensor) else self.correct
        return c / self.count

    def __str__(self):
        return '{:.2f}%'.format(self.accuracy * 100)


class _DeviceAverage(Average):
    def update(self, value, number):
        self.sum = self.sum + value.detach() * number
        self.count += number

    @property
    def average(self):
        s = self.sum.item() if isinstance(self.sum, torch.Tensor) else self.sum
        return s / self.count


def _loss_fn(output, label):
    return ops.cross_entropy(output, label)


class Trainer(object):
    def __init__(self, net, optimizer, train_loader, test_loader, device, distributed, do_eval,
                 manual_average: bool = False, autocast_dtype=None):
        self.net = net
        self.optimizer = optimizer
        self.train_loader = train_loader
        self.test_loader = test_loader
        self.device = device
        self.distributed = distributed
        self.do_eval = do_eval
        self.manual_average = manual_average    # reference path: per-parameter all-reduce after backward
        # mixed precision (``--dtype bf16``): forward + loss under torch.autocast, fp32 parameters,
        # gradients and optimizer state (the loss itself is computed from fp32 logits)
        self.autocast_dtype = autocast_dtype
        self.printer = print

    def _forward(self, data, label):
        if self.autocast_dtype is None:
            output = self.net(data)
            return output, _loss_fn(output, label)
        with torch.autocast(device_type=self.device.type, dtype=self.autocast_dtype):
            output = self.net(data)
        output = output.float()
        return output, _loss_fn(output, label)

    def fit(self, epochs, start_epoch: int = 0):
        """Epochs ``start_epoch+1 .. epochs`` (a resumed run passes the checkpoint's epoch, so the
        sampler's ``set_epoch`` and the printed ``e/E`` use the absolute epoch)."""
        for epoch in range(start_epoch + 1, epochs + 1):
            if hasattr(self.train_loader.sampler, "set_epoch") and getattr(self, "set_epoch", False):
                self.train_loader.sampler.set_epoch(epoch)
            train_loss, train_acc = self.train()
            if (self.do_eval or epoch == epochs):
                test_loss, test_acc = self.evaluate()
            else:
                test_loss, test_acc = 0, 0

            self.printer(
                'Epoch: {}/{},'.format(epoch, epochs),
                'train loss: {}, train acc: {},'.format(train_loss, train_acc),
                'test loss: {}, test acc: {}.'.format(test_loss, test_acc))

    def train(self):
        train_loss = _DeviceAverage()
        train_acc = Accuracy()

        self.net.train()

        for data, label in self.train_loader:
            data = data.to(self.device)
            label = label.to(self.device)

            with prof.range("forward"):
                output, loss = self._forward(data, label)

            self.optimizer.zero_grad()
            with prof.range("backward"):
                loss.backward()
            if self.distributed and self.manual_average:
                with prof.range("average_gradients"):
                    self.average_gradients()
            with prof.range("optimizer"):
                self.optimizer.step()

            train_loss.update(loss, data.size(0))
            train_acc.update(output, label)

        return train_loss, train_acc

    def evaluate(self):
        test_loss = _DeviceAverage()
        test_acc = Accuracy()

        self.net.eval()

        with torch.no_grad():
            for data, label in self.test_loader:
                data = data.to(self.device)
                label = label.to(self.device)

                output, loss = self._forward(data, label)

                test_loss.update(loss, data.size(0))
                test_acc.update(output, label)

        return test_loss, test_acc

    def average_gradients(self):
        world_size = dist.get_world_size()

        for p in self.net.parameters():
            dist.all_reduce(p.grad.data, op=dist.ReduceOp.SUM)
            p.grad.data /= float(world_size)


class FusedTrainer(object):
    """Same interface/prints as ``Trainer`` over the fused LeNet engine."""

    def __init__(self, engine, train_set, test_set, sampler, do_eval, use_graph: bool = True, set_epoch=False):
        self.engine = engine
        self.train_set = train_set
        self.test_set = test_set
        self.sampler = sampler
        self.do_eval = do_eval
        self.use_graph = use_graph
        self.set_epoch = set_epoch
        self.printer = print
        engine.bind_dataset(train_set.images, train_set.labels)

    def fit(self, epochs, start_epoch: int = 0):
        for epoch in range(start_epoch + 1, epochs + 1):
            if self.set_epoch and hasattr(self.sampler, "set_epoch"):
                self.sampler.set_epoch(epoch)
            train_loss, train_acc = self.train()
            if self.do_eval or epoch == epochs:
                test_loss, test_acc = self.evaluate()
            else:
                test_loss, test_acc = 0, 0
            self.printer(
                'Epoch: {}/{},'.format(epoch, epochs),
                'train loss: {}, train acc: {},'.format(train_loss, train_acc),
                'test loss: {}, test acc: {}.'.format(test_loss, test_acc))

    def check_comm_health(self):
        """Raise if the engine's communication path failed (xGMI peer barrier time-out, RCCL error).

        A timed-out peer barrier poisons the peer protocol on purpose: later all-reduces skip their
        barriers and would reduce stale data, so replicas would diverge silently.  Raising makes the
        rank exit non-zero and the launcher tear the gang down instead."""
        comm = getattr(self.engine, "comm", None)
        if comm is None or not hasattr(comm, "health"):
            return
        h = comm.health()
        if h:
            raise RuntimeError(f"data-parallel communication failed: {h}")

    def train(self):
        self.engine.set_epoch_indices(self.sampler.indices_tensor())
        self.engine.run_epoch(use_graph=self.use_graph)
        loss_sum, correct, n = self.engine.read_meters()     # synchronises: the epoch's comm is done
        self.check_comm_health()
        a, acc = Average(), Accuracy()
        a.sum, a.count = loss_sum, n
        acc.correct, acc.count = correct, n
        return a, acc

    def evaluate(self):
        loss_sum, correct, n = self.engine.evaluate(self.test_set.images, self.test_set.labels)
        a, acc = Average(), Accuracy()
        a.sum, a.count = loss_sum, n
        acc.correct, acc.count = correct, n
        return a, acc
