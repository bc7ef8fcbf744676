"""pytorch_distributed_example_amd — an MI355X-native (gfx950 / CDNA4) data-parallel training framework.

Capabilities of dblakely/pytorch-distributed-example (toy all-reduce loop, manual-DP CNN trainer)
re-designed for MI355X: hand-written HIP kernels (MFMA, LDS tiling) for the model's hot ops, a
C++ runtime (TCP rendezvous store, host TCP collectives, RCCL communicator over xGMI), a
torch.distributed-compatible ``dist`` API, bucketed/overlapped ``DistributedDataParallel``,
torch-identical ``DistributedSampler``, fused optimizers and hipGraph-captured training steps.
"""
__version__ = "0.1.0"

from . import _ext  # noqa: F401
