"""CPU plumbing of the driver-added model configs (GPT-2 small, ResNet-18, MLP): shapes, parameter
counts / names of the standard checkpoints, forward+backward on the PyTorch reference ops."""
import torch

from pytorch_distributed_example_amd.models import MLP, GPTConfig, build_gpt2, build_resnet18


def test_gpt2_small_param_count_and_names():
    m = build_gpt2(dtype=torch.float32)
    # GPT-2 small = 124,439,808 with the 50257 vocab; +47*768 for the 50304 padding
    assert m.num_params() == 124_439_808 + (50304 - 50257) * 768
    names = [n for n, _ in m.named_parameters()]
    assert names[:2] == ["transformer.wte.weight", "transformer.wpe.weight"]
    assert "transformer.h.11.mlp.c_proj.weight" in names and names[-1] == "transformer.ln_f.bias"
    assert dict(m.named_parameters())["transformer.h.0.attn.c_attn.weight"].shape == (2304, 768)


def test_gpt2_tiny_cpu_step():
    cfg = GPTConfig(block_size=32, vocab_size=100, padded_vocab=128, n_layer=2, n_head=2, n_embd=32)
    m = build_gpt2(cfg, dtype=torch.float32)
    idx = torch.randint(0, 100, (2, 32))
    loss = m(idx, idx)
    assert abs(loss.item() - torch.log(torch.tensor(100.0)).item()) < 1.0
    loss.backward()
    assert all(p.grad is not None for p in m.parameters())
    assert m(idx).shape == (2, 32, 100)


def test_resnet18_torchvision_layout():
    m = build_resnet18(dtype=torch.float32)
    assert sum(p.numel() for p in m.parameters()) == 11_689_512
    sd = m.state_dict()
    for k in ("conv1.weight", "bn1.running_mean", "bn1.num_batches_tracked", "layer2.0.downsample.0.weight",
              "layer2.0.downsample.1.weight", "layer4.1.bn2.bias", "fc.weight"):
        assert k in sd, k
    assert len(sd) == 122                      # torchvision resnet18 state_dict entries


def test_resnet18_cpu_step_and_running_stats():
    m = build_resnet18(num_classes=10, dtype=torch.float32)
    x = torch.randn(4, 3, 64, 64)
    out = m(x)
    assert out.shape == (4, 10)
    out.sum().backward()
    assert float(m.bn1.running_mean.abs().sum()) > 0
    assert int(m.bn1.num_batches_tracked) == 1
    m.eval()
    with torch.no_grad():
        assert m(x).shape == (4, 10)


def test_mlp_config():
    m = MLP()
    assert sum(p.numel() for p in m.parameters()) == 784 * 512 + 512 + 512 * 10 + 10
