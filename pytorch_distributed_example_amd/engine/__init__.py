"""Fused, hipGraph-capturable training steps."""
from .lenet import LeNetTrainStep  # noqa: F401
