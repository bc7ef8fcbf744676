"""Model zoo: the reference toy CNN (``Net``) plus the driver-added configs."""
from .lenet import Net, build_net, PARAM_SPECS, NUM_PARAMS  # noqa: F401
from .mlp import MLP  # noqa: F401
from .gpt2 import GPT, GPTConfig, build_gpt2  # noqa: F401
from .resnet import ResNet, build_resnet18  # noqa: F401
