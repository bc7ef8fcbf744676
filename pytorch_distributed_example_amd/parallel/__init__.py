"""Data parallelism: flat bucketed gradient storage and DistributedDataParallel."""
from .ddp import DistributedDataParallel, average_gradients, tune_bucket_cap  # noqa: F401
from .flat import FlatLayout, reverse_order_buckets, shared_flat  # noqa: F401

DDP = DistributedDataParallel
