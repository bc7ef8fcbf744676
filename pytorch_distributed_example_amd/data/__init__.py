"""Data: torch-identical samplers, device-resident synthetic datasets, device batch loader."""
from .sampler import DistributedSampler, RandomSampler, SequentialSampler  # noqa: F401
from .synthetic import TensorDataset, synthetic_mnist, idx_dataset, synthetic_tokens, synthetic_images, MEAN, STD  # noqa: F401
from .loader import DeviceDataLoader  # noqa: F401
