"""Implicit-GEMM bf16 MFMA convolutions (csrc/kernels/conv.hip) vs a PyTorch fp32 reference of the
same op on the same bf16-rounded operands: fprop, phase-split dgrad (stride 2 incl. 1x1 / stride 2
with its all-zero phases), split-K wgrad, ragged pixel tiles, and the fused BatchNorm partial sums."""
import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_example_amd._ext import kernels
from pytorch_distributed_example_amd.ops.resnet import conv2d_nhwc, igemm_eligible

pytestmark = pytest.mark.gpu
dev = "cuda"

SHAPES = [
    # B, Cin, H, W, Cout, k, stride, pad
    (2, 64, 9, 9, 64, 3, 1, 1),
    (3, 64, 12, 10, 128, 3, 2, 1),
    (2, 64, 8, 8, 128, 1, 2, 0),
    (2, 128, 7, 7, 128, 1, 1, 0),
    (1, 256, 7, 7, 512, 3, 1, 1),
    (5, 128, 13, 11, 256, 3, 2, 1),
    (4, 64, 56, 56, 64, 3, 1, 1),      # ResNet-18 layer1 geometry
    (2, 512, 7, 7, 512, 3, 1, 1),      # layer4
    # halo-tiled stride-1 3x3 kernel (k_hconv): layer2 / layer3 geometry, partial row tiles, odd widths
    (2, 128, 28, 28, 128, 3, 1, 1),
    (2, 256, 14, 14, 256, 3, 1, 1),
    (3, 64, 17, 23, 128, 3, 1, 1),
    (2, 128, 20, 15, 64, 3, 1, 1),
    (3, 64, 17, 20, 64, 3, 1, 1),      # halo-tiled layer1 wgrad with a ragged last row tile
]


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def max_rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


@pytest.mark.parametrize("B,C,H,W,N,k,s,p", SHAPES)
def test_conv_fwd_bwd(B, C, H, W, N, k, s, p):
    torch.manual_seed(B * 1000 + C + k)
    x = cl(torch.randn(B, C, H, W, device=dev).to(torch.bfloat16)).requires_grad_()
    w = cl((torch.randn(N, C, k, k, device=dev) / (C * k * k) ** 0.5).to(torch.bfloat16)).requires_grad_()
    assert igemm_eligible(x, w, s, p)
    y = conv2d_nhwc(x, w, s, p)
    assert y.is_contiguous(memory_format=torch.channels_last)
    dy = cl(torch.randn_like(y))
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    yr = F.conv2d(xr, wr, None, s, p)
    yr.backward(dy.float())
    assert y.shape == yr.shape
    assert max_rel(y, yr) < 1e-2
    assert max_rel(x.grad, xr.grad) < 1e-2
    assert max_rel(w.grad, wr.grad) < 1e-2
    assert x.grad.is_contiguous(memory_format=torch.channels_last)


def test_conv_exact_integer_data():
    """Small integers are exact in bf16 and in fp32 accumulation: any indexing slip shows exactly."""
    torch.manual_seed(7)
    B, C, H, W, N = 3, 64, 6, 5, 128
    x = cl(torch.randint(-1, 2, (B, C, H, W), device=dev).to(torch.bfloat16)).requires_grad_()
    w = cl(torch.randint(-1, 2, (N, C, 3, 3), device=dev).to(torch.bfloat16)).requires_grad_()
    y = conv2d_nhwc(x, w, 2, 1)
    dy = cl(torch.randint(-1, 2, y.shape, device=dev).to(torch.bfloat16))
    y.backward(dy)
    xr, wr = x.detach().double().cpu().requires_grad_(), w.detach().double().cpu().requires_grad_()
    yr = F.conv2d(xr, wr, None, 2, 1)
    yr.backward(dy.double().cpu())
    assert torch.equal(y.double().cpu(), yr)
    assert torch.equal(x.grad.double().cpu(), xr.grad)
    assert torch.equal(w.grad.double().cpu(), wr.grad)


@pytest.mark.parametrize("B,C,H,W,N", [(2, 128, 28, 28, 128), (2, 256, 14, 14, 256), (3, 64, 17, 23, 128),
                                       (2, 128, 20, 15, 64)])
def test_hconv_tap_loop_forms_identical(B, C, H, W, N, monkeypatch):
    """k_hconv's two tap-loop forms (PDE_HCONV_V=0: fragment addresses hoisted out of the channel loop;
    1: formed per tap, the default) run the same MFMA sequence: bit-identical fprop and dgrad, and
    exact on integer data."""
    torch.manual_seed(C + W)
    x = cl(torch.randint(-2, 3, (B, C, H, W), device=dev).to(torch.bfloat16))
    w = cl(torch.randint(-1, 2, (N, C, 3, 3), device=dev).to(torch.bfloat16))
    dy = cl(torch.randint(-1, 2, (B, N, H, W), device=dev).to(torch.bfloat16))
    got = []
    for v in ("0", "1"):
        monkeypatch.setenv("PDE_HCONV_V", v)
        xv = x.clone().requires_grad_()
        y = conv2d_nhwc(xv, w, 1, 1)
        y.backward(dy)
        got.append((y.detach(), xv.grad))
    assert torch.equal(got[0][0], got[1][0]) and torch.equal(got[0][1], got[1][1])
    yr = F.conv2d(x.double().cpu(), w.double().cpu(), None, 1, 1)
    assert torch.equal(got[1][0].double().cpu(), yr)


@pytest.mark.parametrize("B,H,W", [(4, 56, 56), (3, 17, 20)])
def test_hconv64_read_forms_identical(B, H, W, monkeypatch):
    """The persistent layer-1 halo conv (k_hconv64) with a tap's fragments read ahead of its MFMAs
    (default) and interleaved with them (PDE_HC64_PIPE=0): bit-identical fprop and dgrad, exact on
    integer data."""
    torch.manual_seed(H + W)
    x = cl(torch.randint(-2, 3, (B, 64, H, W), device=dev).to(torch.bfloat16))
    w = cl(torch.randint(-1, 2, (64, 64, 3, 3), device=dev).to(torch.bfloat16))
    dy = cl(torch.randint(-1, 2, (B, 64, H, W), device=dev).to(torch.bfloat16))
    got = []
    for v in ("0", "1"):
        monkeypatch.setenv("PDE_HC64_PIPE", v)
        xv = x.clone().requires_grad_()
        y = conv2d_nhwc(xv, w, 1, 1)
        y.backward(dy)
        got.append((y.detach(), xv.grad))
    assert torch.equal(got[0][0], got[1][0]) and torch.equal(got[0][1], got[1][1])
    yr = F.conv2d(x.double().cpu(), w.double().cpu(), None, 1, 1)
    assert torch.equal(got[1][0].double().cpu(), yr)


@pytest.mark.parametrize("N", [64, 128])
@pytest.mark.parametrize("B,H,W", [(3, 10, 9), (2, 12, 20), (2, 9, 56), (24, 56, 56)])
def test_conv_fprop_bn_stats(N, B, H, W):
    """BN statistics partials from the conv epilogue (implicit GEMM for narrow images, the halo-tiled
    kernel for W >= 14): one row per M tile of whichever kernel ran (one per block of the persistent
    k_hconv64, which at B=24 walks 336 row tiles on <= 256 blocks), folding to the batch sums."""
    torch.manual_seed(11)
    K = kernels()
    C = 64
    x = cl(torch.randn(B, C, H, W, device=dev).to(torch.bfloat16))
    w = cl((torch.randn(N, C, 3, 3, device=dev) / 24).to(torch.bfloat16))
    y = cl(torch.empty(B, N, H, W, device=dev, dtype=torch.bfloat16))
    nblk = K.conv_stats_rows(x, w, 1, 1)
    stats = torch.empty(nblk * 2 * N, device=dev)
    K.conv_fprop(x, w, y, stats, 1, 1)
    st = stats.view(nblk, 2, N).sum(0)
    assert torch.allclose(y.float(), F.conv2d(x.float(), w.float(), None, 1, 1), rtol=2e-2, atol=2e-2)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, N)
    assert torch.allclose(st[0], yf.sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(st[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-3)


# ---------------------------------------------------------------------------------------------- stem
from pytorch_distributed_example_amd.ops.resnet import stem_eligible  # noqa: E402


@pytest.mark.parametrize("B,H,W", [(2, 224, 224), (3, 64, 64), (2, 37, 51), (1, 10, 7)])
def test_stem_conv_fwd_bwd(B, H, W):
    """7x7 / s2 / p3 stem kernel (csrc/kernels/stem.hip) vs fp32 conv2d on the same bf16 operands."""
    torch.manual_seed(B * 100 + H + W)
    x = cl(torch.randn(B, 3, H, W, device=dev).to(torch.bfloat16))      # the image: no gradient
    w = cl((torch.randn(64, 3, 7, 7, device=dev) / 147 ** 0.5).to(torch.bfloat16)).requires_grad_()
    assert stem_eligible(x, w, 2, 3)
    y = conv2d_nhwc(x, w, 2, 3)
    assert y.is_contiguous(memory_format=torch.channels_last)
    dy = cl(torch.randn_like(y))
    y.backward(dy)
    xr = x.detach().float()
    wr = w.detach().float().requires_grad_()
    yr = F.conv2d(xr, wr, None, 2, 3)
    yr.backward(dy.float())
    assert y.shape == yr.shape
    assert max_rel(y, yr) < 1e-2
    assert max_rel(w.grad, wr.grad) < 2e-2
    # no input-gradient kernel for the 3-channel stem: asking for one raises (no silent ATen path)
    with pytest.raises(NotImplementedError):
        conv2d_nhwc(x.detach().requires_grad_(), w, 2, 3).backward(dy)


def test_stem_exact_integer_and_stats():
    """Integer data is exact in bf16 / fp32: any tap or padding slip shows; BN partials sum to the
    per-channel (sum, sum of squares) of the bf16 output."""
    torch.manual_seed(3)
    K = kernels()
    B, H, W = 2, 30, 26
    x = cl(torch.randint(-2, 3, (B, 3, H, W), device=dev).to(torch.bfloat16))
    w = cl(torch.randint(-1, 2, (64, 3, 7, 7), device=dev).to(torch.bfloat16))
    y, (part, nblk) = conv2d_nhwc(x, w, 2, 3, with_stats=True)
    yr = F.conv2d(x.double().cpu(), w.double().cpu(), None, 2, 3)
    assert torch.equal(y.double().cpu(), yr)
    assert nblk == K.stem_stats_blocks(B, y.shape[2])
    st = part[: nblk * 128].view(nblk, 2, 64).sum(0).double().cpu()
    yf = yr.permute(0, 2, 3, 1).reshape(-1, 64)
    assert torch.allclose(st[0], yf.sum(0), rtol=1e-6, atol=1e-3)
    assert torch.allclose(st[1], (yf * yf).sum(0), rtol=1e-6, atol=1e-3)


@pytest.mark.parametrize("B,C,H,W,N,k,s,p", [SHAPES[0], SHAPES[1], SHAPES[2]])
def test_conv_dgrad_residual_accumulate(B, C, H, W, N, k, s, p):
    """dgrad with the residual-gradient add in its epilogue: dx = bf16(dgrad) + res, as autograd's
    separate bf16 add would produce."""
    torch.manual_seed(11)
    x = cl(torch.randn(B, C, H, W, device=dev).to(torch.bfloat16))
    w = cl((torch.randn(N, C, k, k, device=dev) / (C * k * k) ** 0.5).to(torch.bfloat16))
    y = conv2d_nhwc(x, w, s, p)
    dy = cl(torch.randn_like(y))
    res = cl(torch.randn_like(x))
    K = kernels()
    wt = torch.empty(w.numel(), device=dev, dtype=w.dtype)
    dx0 = torch.empty_like(x, memory_format=torch.channels_last)
    K.conv_dgrad(dy, w, wt, dx0, s, p)
    dx1 = torch.empty_like(x, memory_format=torch.channels_last)
    K.conv_dgrad(dy, w, wt, dx1, s, p, res)
    assert torch.equal(dx1, (dx0.float() + res.float()).to(torch.bfloat16))


@pytest.mark.parametrize("B,C,H,W,N,k", [
    (4, 64, 56, 56, 64, 3),     # k_hconv64 (layer1)
    (24, 64, 56, 56, 64, 3),    # k_hconv64 over 336 row tiles: one partial row per persistent block
    (40, 128, 28, 28, 128, 3),  # k_hconv<128, 128>, 280 partial rows: the finalize's pre-fold
    (2, 128, 28, 28, 128, 3),   # k_hconv<128, 128> (layer2)
    (3, 64, 17, 23, 128, 3),    # k_hconv<256, 64>, ragged row tiles
    (2, 512, 7, 7, 512, 3),     # k_igemm<128, 128> (layer4)
    (3, 64, 9, 7, 128, 1),      # k_igemm<256, 64>, 1x1
])
def test_conv_dgrad_bn_partials(B, C, H, W, N, k):
    """BN-backward reduction fused into the dgrad epilogue (conv.hip BnbArgs): dx unchanged (bitwise),
    the partials == fp32 sums of d = dx * (bx*scale + shift > 0) and d * xhat, and bn_bwd from the
    pre-summed partials == bn_bwd with its own reduce pass."""
    torch.manual_seed(13)
    K = kernels()
    p = k // 2
    dy = cl(torch.randn(B, N, H, W, device=dev).to(torch.bfloat16))
    w = cl((torch.randn(N, C, k, k, device=dev) / (C * k * k) ** 0.5).to(torch.bfloat16))
    bx = cl((torch.randn(B, C, H, W, device=dev) * 2 + 0.3).to(torch.bfloat16))
    mean = torch.randn(C, device=dev) * 0.1 + 0.3
    rstd = torch.rand(C, device=dev) + 0.5
    gamma = (torch.rand(C, device=dev) + 0.5).to(torch.bfloat16)
    beta = (torch.randn(C, device=dev) * 0.1).to(torch.bfloat16)
    scale = gamma.float() * rstd
    shift = beta.float() - mean * scale
    wt = torch.empty(w.numel(), device=dev, dtype=w.dtype)
    dx0 = torch.empty_like(bx)
    K.conv_dgrad(dy, w, wt, dx0, 1, p)
    rows = K.conv_dgrad_bn_rows(bx, w, 1, p)
    assert rows > 0
    part = torch.full((K.bn_part_rows(rows) * 2 * C,), float("nan"), device=dev)
    dx = torch.empty_like(bx)
    K.conv_dgrad(dy, w, wt, dx, 1, p, wt_ready=True, bn_x=bx, bn_scale=scale, bn_shift=shift, bn_mean=mean,
                 bn_rstd=rstd, bn_part=part)
    assert torch.equal(dx, dx0)
    st = part[: rows * 2 * C].view(rows, 2, C).double().sum(0).cpu()
    xf = bx.permute(0, 2, 3, 1).reshape(-1, C).double().cpu()
    gf = dx.permute(0, 2, 3, 1).reshape(-1, C).double().cpu()
    d = torch.where(xf * scale.double().cpu() + shift.double().cpu() > 0, gf, torch.zeros_like(gf))
    ref_s = d.sum(0)
    ref_q = (d * (xf - mean.double().cpu()) * rstd.double().cpu()).sum(0)
    assert torch.allclose(st[0], ref_s, rtol=1e-4, atol=1e-2 + 1e-5 * d.abs().sum().item() / C)
    assert torch.allclose(st[1], ref_q, rtol=1e-4, atol=1e-2 + 1e-5 * d.abs().sum().item() / C)
    # bn_bwd: pre-summed partials vs the reduce pass
    M = B * H * W
    outs = []
    for pre in (True, False):
        pp = part if pre else torch.empty(K.bn_blocks(M, C) * 2 * C, device=dev)
        coef = torch.empty(3 * C, device=dev)
        dg = torch.empty(C, device=dev, dtype=torch.bfloat16)
        db = torch.empty(C, device=dev, dtype=torch.bfloat16)
        dxx = torch.empty_like(bx)
        K.bn_bwd(dx, None, bx, gamma, mean, rstd, pp, coef, dg, db, dxx, None, True, scale, shift,
                 rows if pre else 0)
        outs.append((dg.float(), db.float(), dxx.float(), coef))
    (g1, b1, x1, c1), (g2, b2, x2, c2) = outs
    assert torch.allclose(g1, g2, rtol=1e-2, atol=1e-2 * g2.abs().max().item())
    assert torch.allclose(b1, b2, rtol=1e-2, atol=1e-2 * b2.abs().max().item())
    assert torch.allclose(c1, c2, rtol=1e-3, atol=1e-4 * c2.abs().max().item())
    assert max_rel(x1, x2) < 1e-2


@pytest.mark.parametrize("B,C,H,W,N", [(4, 64, 56, 56, 128), (3, 128, 14, 14, 256), (2, 64, 9, 7, 64)])
def test_conv_dgrad_fused_downsample(B, C, H, W, N):
    """3x3 / s2 / p1 dgrad with a 1x1 / s2 / p0 downsample's input gradient as extra K stages of the
    even-pixel phase == fp32 sum of both input gradients (one bf16 rounding instead of two)."""
    torch.manual_seed(12)
    x = cl(torch.randn(B, C, H, W, device=dev).to(torch.bfloat16))
    w = cl((torch.randn(N, C, 3, 3, device=dev) / (C * 9) ** 0.5).to(torch.bfloat16))
    wd = cl((torch.randn(N, C, 1, 1, device=dev) / C ** 0.5).to(torch.bfloat16))
    y = conv2d_nhwc(x, w, 2, 1)
    dy = cl(torch.randn_like(y))
    dyd = cl(torch.randn_like(y))
    K = kernels()
    wt = torch.empty(w.numel(), device=dev, dtype=w.dtype)
    wdt = torch.empty(wd.numel(), device=dev, dtype=w.dtype)
    dx = torch.empty_like(x, memory_format=torch.channels_last)
    K.conv_dgrad(dy, w, wt, dx, 2, 1, None, dyd, wd, wdt)
    xr = x.float().requires_grad_()
    (F.conv2d(xr, w.float(), None, 2, 1) * dy.float()).sum().add_(
        (F.conv2d(xr, wd.float(), None, 2, 0) * dyd.float()).sum()).backward()
    err = (dx.float() - xr.grad).abs().max().item()
    assert err <= 1e-2 * xr.grad.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("C,H,N,k,s,p", [(64, 56, 128, 3, 2, 1), (128, 28, 128, 3, 1, 1), (128, 28, 256, 3, 2, 1),
                                         (256, 14, 256, 3, 1, 1), (256, 14, 512, 3, 2, 1), (512, 7, 512, 3, 1, 1),
                                         (64, 56, 128, 1, 2, 0)])
def test_wgrad_split_fits_one_block_round(C, H, N, k, s, p):
    """The split-K wgrad grid (tiles x splits) of every ResNet-18 layer-2..4 geometry at B=256 stays
    within one round of co-resident blocks (2 per CU): a ceil-rounded split count launched 513-576
    blocks, and the few past the round ran as a tail as long as a whole block
    (profiles/r3_models/wgrad_blocks_sweep.jsonl)."""
    K = kernels()
    B = 256
    x = torch.empty(B, C, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.empty(N, C, k, k, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    splits = K.conv_wgrad_splits(x, w, s, p)
    BM = 128 if N % 128 == 0 else 64
    tiles = (N // BM) * ((k * k * C + 127) // 128)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    assert 1 <= splits and splits * tiles <= 2 * ncu
    if k == 3:
        assert splits * tiles > ncu      # and fills at least one block per CU
