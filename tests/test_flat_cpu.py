"""FlatLayout: channels-last 4-D parameters keep their layout in flat storage, and the grad-slot
protocol (ops write a parameter's gradient straight into its flat slot; autograd adopts it)."""
import torch

from pytorch_distributed_example_amd.parallel.flat import FlatLayout, flat_grad_slot


def test_channels_last_slot_roundtrip():
    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(8, 4, 3, 3).contiguous(memory_format=torch.channels_last))
    b = torch.nn.Parameter(torch.randn(8))
    ref = w.detach().clone()
    layout = FlatLayout([("w", tuple(w.shape)), ("b", (8,))], [["w", "b"]])
    fp, fg = layout.bind({"w": w, "b": b})
    assert w.is_contiguous(memory_format=torch.channels_last) and not w.is_contiguous()
    assert torch.equal(w.detach(), ref)
    # physical order of the slot is [N][H][W][C]
    assert torch.equal(fp[: w.numel()], ref.permute(0, 2, 3, 1).reshape(-1))
    assert w.grad.stride() == w.stride() and w.grad.data_ptr() == fg.data_ptr()


def test_grad_slot_adopted_by_autograd():
    class Scale(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            ctx.save_for_backward(x, w)
            return x * w

        @staticmethod
        def backward(ctx, g):
            x, w = ctx.saved_tensors
            dw = flat_grad_slot(w)
            val = (g * x).sum(0)
            if dw is None:
                return g * w, val
            dw.copy_(val)
            return g * w, dw

    w = torch.nn.Parameter(torch.randn(16))
    layout = FlatLayout([("w", (16,))], [["w"]])
    fp, fg = layout.bind({"w": w})
    x = torch.randn(5, 16)
    w.grad = None
    Scale.apply(x, w).sum().backward()
    assert w.grad.data_ptr() == fg.data_ptr()              # written in place, no copy
    assert torch.allclose(w.grad, x.sum(0))
    Scale.apply(x, w).sum().backward()                       # accumulation falls back to a new tensor
    assert torch.allclose(w.grad, 2 * x.sum(0))
