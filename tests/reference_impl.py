"""Plain-PyTorch fp32/fp64 references used by the numerics tests (stock ATen ops only)."""
import torch
import torch.nn as nn
import torch.nn.functional as F


class TorchNet(nn.Module):
    """Stock torch.nn re-statement of the reference model (mnist/main.py:130-147) for parity checks."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 20, 5, 1)
        self.conv2 = nn.Conv2d(20, 50, 5, 1)
        self.fc1 = nn.Linear(800, 500)
        self.fc2 = nn.Linear(500, 10)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.conv1(x)), 2, 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2, 2)
        x = F.relu(self.fc1(x.view(-1, 800)))
        return F.log_softmax(self.fc2(x), dim=1)


def torch_twin(net, dtype=torch.float64, device="cpu"):
    ref = TorchNet().to(device=device, dtype=dtype)
    ref.load_state_dict({k: v.detach().to(device=device, dtype=dtype) for k, v in net.state_dict().items()})
    return ref


def ref_step_grads(ref, x, y):
    ref.zero_grad(set_to_none=True)
    out = ref(x)
    loss = F.cross_entropy(out, y)
    loss.backward()
    return out.detach(), loss.detach(), {n: p.grad.detach().clone() for n, p in ref.named_parameters()}
