"""Fused optimizers (one HIP launch per step over a flat buffer), torch.optim-compatible state."""
from .fused import SGD, Adam, AdamW  # noqa: F401
from .master import AdamWMaster, SGDMaster  # noqa: F401
