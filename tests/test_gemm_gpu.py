"""Own bf16 MFMA GEMM (csrc/kernels/gemm.hip) vs plain PyTorch fp32 references: every tile
configuration, ragged M / N tiles, split-K with the fused bias gradient, and the fused bias /
GELU / GELU-backward epilogues, at small shapes and at the GPT-2 projection shapes."""
import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_example_amd._ext import kernels
from pytorch_distributed_example_amd.ops import gemm as G

pytestmark = pytest.mark.gpu
dev = "cuda"
CFGS = list(range(23))


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def _bf(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dev, torch.bfloat16)


def test_tiles_and_cfgs():
    K = kernels()
    assert K.gemm_num_cfgs() == 23
    assert [tuple(K.gemm_tile(c)) for c in CFGS] == [(256, 192), (256, 128), (128, 128), (256, 256), (128, 128),
                                                     (256, 256), (256, 192), (256, 128), (128, 128), (256, 192),
                                                     (256, 192), (256, 256), (256, 256), (256, 128), (256, 192),
                                                     (256, 256), (256, 192), (256, 256), (256, 256), (256, 256), (256, 256), (256, 192), (256, 192)]
    assert K.gemm_splits(16384, 8) == 8 and K.gemm_splits(192, 8) == 3


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("M,N,K", [(300, 200, 192), (64, 8, 64), (513, 776, 320)])
def test_fprop_bias(cfg, M, N, K):
    x, w, b = _bf(M, K, seed=1), _bf(N, K, scale=0.05, seed=2), _bf(N, seed=3)
    y = G.fprop(x, w, b, cfg=cfg)
    ref = F.linear(x.float(), w.float(), b.float())
    assert y.shape == (M, N)
    assert rel_err(y, ref) < 1e-2
    y0 = G.fprop(x, w, None, cfg=cfg)
    assert rel_err(y0, x.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("cfg", CFGS)
def test_fprop_gelu(cfg):
    M, N, K = 520, 392, 256
    x, w, b = _bf(M, K, seed=4), _bf(N, K, scale=0.06, seed=5), _bf(N, scale=0.5, seed=6)
    act, dgelu = G.fprop(x, w, b, gelu=True, cfg=cfg)
    rp = F.linear(x.float(), w.float(), b.float()).requires_grad_()
    ref = F.gelu(rp, approximate="tanh")
    ref.backward(torch.ones_like(ref))
    # gelu and gelu' of the fp32 accumulator rounded once to bf16 (the pre-activation is never stored)
    assert rel_err(act, ref) < 2e-2
    assert rel_err(dgelu, rp.grad) < 2e-2


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("M,N,K", [(300, 200, 192), (257, 392, 128)])
def test_dgrad(cfg, M, N, K):
    # dx [M, N] = dy [M, K] . w [K, N]  (w is the nn.Linear weight [out=K][in=N])
    dy, w = _bf(M, K, seed=7), _bf(K, N, scale=0.05, seed=8)
    dx = G.dgrad(dy, w, cfg=cfg)
    assert rel_err(dx, dy.float() @ w.float()) < 1e-2
    pre = _bf(M, N, seed=9).float().requires_grad_()
    F.gelu(pre, approximate="tanh").backward(torch.ones_like(pre))
    dgelu = pre.grad.to(torch.bfloat16)                  # gelu'(pre) as the forward epilogue saves it
    dxg = G.dgrad(dy, w, dgelu=dgelu, cfg=cfg)
    assert rel_err(dxg, dx.float() * dgelu.float()) < 1e-2


@pytest.mark.parametrize("cfg", [9, 16, 17, 18, 19])
@pytest.mark.parametrize("splits", [2, 4])
def test_dgrad_split_k(cfg, splits):
    """Split-K dgrad (fp32 slabs + the reduction kernel, with the loss-gradient scale folded there):
    the LM-head form, a deep reduction onto few output tiles; ragged M / N and a K % 64 tail."""
    M, N, K = 1000, 392, 5000
    dy, w = _bf(M, K, seed=80), _bf(K, N, scale=0.02, seed=81)
    s = torch.tensor([0.37], device=dev)
    ref = dy.float() @ w.float()
    assert rel_err(G.dgrad(dy, w, cfg=cfg, splits=splits), ref) < 1e-2
    assert rel_err(G.dgrad(dy, w, cfg=cfg, splits=splits, scale=s), ref * 0.37) < 1e-2


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("splits", [1, 3, 8])
def test_wgrad_split_bias(cfg, splits):
    T, N, K = 1024, 392, 200
    dy, x = _bf(T, N, seed=10), _bf(T, K, seed=11)
    dw, db = G.wgrad(dy, x, want_db=True, cfg=cfg, splits=splits)
    assert rel_err(dw, dy.float().t() @ x.float()) < 1e-2
    assert rel_err(db, dy.float().sum(0)) < 1e-2
    dw2, db2 = G.wgrad(dy, x, cfg=cfg, splits=splits)
    assert db2 is None and torch.equal(dw, dw2)


@pytest.mark.parametrize("kind,M,N,K", [
    ("fprop", 4096, 2304, 768), ("fprop", 4096, 768, 3072), ("dgrad", 4096, 768, 3072),
    ("wgrad", 3072, 768, 4096), ("fprop", 2048, 50304, 768), ("dgrad", 2048, 768, 50304),
    ("wgrad", 50304, 768, 2048)])
def test_gpt2_shapes(kind, M, N, K):
    """GPT-2 projection / LM-head shapes (tokens reduced to 2-4k to keep the fp32 reference cheap)."""
    if kind == "fprop":
        x, w, b = _bf(M, K, seed=12), _bf(N, K, scale=0.03, seed=13), _bf(N, seed=14)
        out, ref = G.fprop(x, w, b), F.linear(x.float(), w.float(), b.float())
    elif kind == "dgrad":
        dy, w = _bf(M, K, seed=15), _bf(K, N, scale=0.03, seed=16)
        out, ref = G.dgrad(dy, w), dy.float() @ w.float()
    else:
        dy, x = _bf(K, M, scale=0.1, seed=17), _bf(K, N, seed=18)
        out, _ = G.wgrad(dy, x)
        ref = dy.float().t() @ x.float()
    assert rel_err(out, ref) < 1e-2


def test_wgrad_into_slot_and_strided_reuse():
    """wgrad writes into a given (flat-buffer) slot; scratch slabs are reused across shapes."""
    flat = torch.zeros(392 * 200 + 64, device=dev, dtype=torch.bfloat16)
    slot = flat[64:].view(392, 200)
    dy, x = _bf(2048, 392, seed=19), _bf(2048, 200, seed=20)
    G.wgrad(dy, x, dw=slot)
    assert rel_err(slot, dy.float().t() @ x.float()) < 1e-2
    assert torch.count_nonzero(flat[:64]) == 0


@pytest.mark.parametrize("cfg", CFGS)
def test_k_tail(cfg):
    """K % 64 != 0: K-contiguous operands mask the chunks past K, transposed ones end at row K (wgrad
    over a token count that is not even a multiple of 8)."""
    x, w, b = _bf(300, 200, seed=21), _bf(392, 200, scale=0.05, seed=22), _bf(392, seed=23)
    assert rel_err(G.fprop(x, w, b, cfg=cfg), F.linear(x.float(), w.float(), b.float())) < 1e-2
    dy, w2 = _bf(300, 1000, seed=24), _bf(1000, 392, scale=0.05, seed=25)
    assert rel_err(G.dgrad(dy, w2, cfg=cfg), dy.float() @ w2.float()) < 1e-2
    for T in (37, 300):
        dy3, x3 = _bf(T, 392, seed=26), _bf(T, 200, seed=27)
        dw, db = G.wgrad(dy3, x3, want_db=True, cfg=cfg, splits=2)
        assert rel_err(dw, dy3.float().t() @ x3.float()) < 1e-2
        assert rel_err(db, dy3.float().sum(0)) < 1e-2


@pytest.mark.parametrize("cfg", [14, 15, 16, 17, 19, 20])
@pytest.mark.parametrize("M,N,K", [(8200, 1544, 192), (4100, 3080, 1000)])
def test_persistent_multi_tile(cfg, M, N, K):
    """Persistent configs with more tiles than CUs (each block walks several tiles, a tile's stores in
    flight under the next tile's first K stage): ragged M / N edges, a short K and a K % 64 tail; bias,
    GELU and GELU backward epilogues."""
    x, w, b = _bf(M, K, seed=30), _bf(N, K, scale=0.05, seed=31), _bf(N, seed=32)
    y = G.fprop(x, w, b, cfg=cfg)
    rp = F.linear(x.float(), w.float(), b.float())
    assert rel_err(y, rp) < 1e-2
    act, dgelu = G.fprop(x, w, b, gelu=True, cfg=cfg)
    rq = rp.clone().requires_grad_()
    ref = F.gelu(rq, approximate="tanh")
    ref.backward(torch.ones_like(ref))
    assert rel_err(act, ref) < 2e-2 and rel_err(dgelu, rq.grad) < 2e-2
    dy, w2 = _bf(M, K, seed=33), _bf(K, N, scale=0.05, seed=34)
    dx = G.dgrad(dy, w2, cfg=cfg)
    rd = dy.float() @ w2.float()
    assert rel_err(dx, rd) < 1e-2
    dxg = G.dgrad(dy, w2, dgelu=dgelu, cfg=cfg)
    assert rel_err(dxg, rd * dgelu.float()) < 1e-2


@pytest.mark.parametrize("M,N,K", [(4100, 2312, 768), (1000, 3072, 3072), (256, 256, 64), (700, 520, 1216)])
def test_gemm8p_fprop(M, N, K):
    """cfg 18, the 8-phase fprop loop (four half-tile regions per K-tile buffer restaged as soon as their
    readers are two phases back, counted vmcnt): ragged M / N tiles, one K-tile, odd K-tile counts, the
    GPT-2 c_attn / mlp shapes; bias and GELU epilogues against fp32 torch."""
    x, w, b = _bf(M, K, seed=40), _bf(N, K, scale=0.03, seed=41), _bf(N, seed=42)
    rp = F.linear(x.float(), w.float(), b.float())
    assert rel_err(G.fprop(x, w, b, cfg=18), rp) < 1e-2
    act, dgelu = G.fprop(x, w, b, gelu=True, cfg=18)
    rq = rp.clone().requires_grad_()
    ref = F.gelu(rq, approximate="tanh")
    ref.backward(torch.ones_like(ref))
    assert rel_err(act, ref) < 2e-2 and rel_err(dgelu, rq.grad) < 2e-2
    # bit-identical to the 2-phase 16x16x32 loop at the same tile (same k order per accumulator)
    assert torch.equal(G.fprop(x, w, b, cfg=18), G.fprop(x, w, b, cfg=17))


@pytest.mark.parametrize("M,N,K", [(4100, 776, 2304), (1000, 3072, 768), (300, 200, 192)])
def test_gemm8p_dgrad(M, N, K):
    """cfg 18 with the transposed B operand (dgrad: two B regions of two 64-column images, vmcnt(6)):
    plain and GELU-backward epilogues vs fp32 torch, bit-identical to cfg 17."""
    dy, w = _bf(M, K, seed=43), _bf(K, N, scale=0.03, seed=44)
    dx = G.dgrad(dy, w, cfg=18)
    assert rel_err(dx, dy.float() @ w.float()) < 1e-2
    assert torch.equal(dx, G.dgrad(dy, w, cfg=17))
    dgelu = _bf(M, N, seed=45)
    dxg = G.dgrad(dy, w, dgelu=dgelu, cfg=18)
    assert torch.equal(dxg, G.dgrad(dy, w, dgelu=dgelu, cfg=17))


@pytest.mark.parametrize("T,N,K,splits", [(4096, 2304, 768, 3), (2048, 768, 3072, 2), (1000, 392, 200, 1),
                                          (300, 520, 264, 2)])
def test_gemm8p_wgrad(T, N, K, splits):
    """cfg 18 with both operands transposed (split-K fp32 slabs, the bias gradient from the ones-MFMA
    spread over waves 0-3): dW and db vs fp32 torch and bit-identical to cfg 17; token counts that are
    not multiples of 64 end at the operands' buffer bounds."""
    dy, x = _bf(T, N, scale=0.1, seed=46), _bf(T, K, seed=47)
    dw, db = G.wgrad(dy, x, want_db=True, cfg=18, splits=splits)
    assert rel_err(dw, dy.float().t() @ x.float()) < 1e-2
    assert rel_err(db, dy.float().sum(0)) < 1e-2
    dw17, db17 = G.wgrad(dy, x, want_db=True, cfg=17, splits=splits)
    assert torch.equal(dw, dw17) and torch.equal(db, db17)


@pytest.mark.parametrize("M,N,K", [(16384, 2304, 768), (9000, 3072, 768), (4100, 776, 1536), (300, 200, 64),
                                   (20000, 2056, 128)])
def test_gemm8pp_persistent_bit_identical(M, N, K):
    """cfg 19, the 8-phase loop in a persistent block per CU (the next tile's prologue DMA issued before
    this tile's stores; round 6: the first K-tile's counted waits no longer treat those stores as still
    in flight, profiles/r6_gemm/): bit-identical to cfg 18 over many tiles per block, ragged edges, one-
    and two-K-tile shapes; fprop (bias, GELU) and dgrad (plain, GELU backward).  Each form runs 3 times
    (a race shows as run-to-run differences)."""
    x, w, b = _bf(M, K, seed=50), _bf(N, K, scale=0.03, seed=51), _bf(N, seed=52)
    y = G.fprop(x, w, b, cfg=19)
    assert rel_err(y, F.linear(x.float(), w.float(), b.float())) < 1e-2
    y18 = G.fprop(x, w, b, cfg=18)
    a18, d18 = G.fprop(x, w, b, gelu=True, cfg=18)
    dy, w2 = _bf(M, K, seed=53), _bf(K, N, scale=0.03, seed=54)
    dg = _bf(M, N, seed=55)
    x18, xg18 = G.dgrad(dy, w2, cfg=18), G.dgrad(dy, w2, dgelu=dg, cfg=18)
    for _ in range(3):
        assert torch.equal(G.fprop(x, w, b, cfg=19), y18)
        a19, d19 = G.fprop(x, w, b, gelu=True, cfg=19)
        assert torch.equal(a19, a18) and torch.equal(d19, d18)
        assert torch.equal(G.dgrad(dy, w2, cfg=19), x18)
        assert torch.equal(G.dgrad(dy, w2, dgelu=dg, cfg=19), xg18)


@pytest.mark.parametrize("cfg", [19, 20])
def test_persistent_dgrad_ragged_rows_regression(cfg):
    """The round-5 failure: cfg 19 (and 20) dgrad at M = 9000 (a ragged last row tile, the blocks' second
    tile) returned wrong values in that tile in 2-4 of 5 repeats; reproduced in round 6 with the old
    tile-boundary wait (tools/gemm_store_order.py mode 1).  10 repeats, plain and (cfg 19) GELU-backward,
    bit-identical to cfg 18."""
    M, N, K = 9000, 3072, 768
    dy, w2 = _bf(M, K, seed=56), _bf(K, N, scale=0.03, seed=57)
    dg = _bf(M, N, seed=58)
    ref, refg = G.dgrad(dy, w2, cfg=18), G.dgrad(dy, w2, dgelu=dg, cfg=18)
    for _ in range(10):
        assert torch.equal(G.dgrad(dy, w2, cfg=cfg), ref)
        if cfg == 19:
            assert torch.equal(G.dgrad(dy, w2, dgelu=dg, cfg=cfg), refg)


@pytest.mark.parametrize("M,N,K", [(16384, 2304, 768), (9000, 3072, 768), (4100, 776, 1536), (20000, 2056, 128),
                                   (300, 200, 256), (16384, 768, 3072)])
def test_gemm8pc_continuous_bit_identical(M, N, K):
    """cfg 20: one K-tile stream per persistent block (the next tile's first K-tiles issued as ordinary
    look-ahead slots), register epilogue merging block pairs across lanes: bit-identical to cfg 18 for
    fprop (with and without bias) and plain dgrad (also with a loss-gradient scale), over many tiles
    per block and ragged edges; every form twice."""
    x, w, b = _bf(M, K, seed=60), _bf(N, K, scale=0.03, seed=61), _bf(N, seed=62)
    y = G.fprop(x, w, b, cfg=20)
    assert rel_err(y, F.linear(x.float(), w.float(), b.float())) < 1e-2
    y18 = G.fprop(x, w, b, cfg=18)
    n18 = G.fprop(x, w, None, cfg=18)
    a18, d18 = G.fprop(x, w, b, gelu=True, cfg=18)
    dy, w2 = _bf(M, K, seed=63), _bf(K, N, scale=0.03, seed=64)
    s = torch.tensor([0.37], device=dev)
    x18, xs18 = G.dgrad(dy, w2, cfg=18), G.dgrad(dy, w2, cfg=18, scale=s)
    for _ in range(2):
        assert torch.equal(G.fprop(x, w, b, cfg=20), y18)
        assert torch.equal(G.fprop(x, w, None, cfg=20), n18)
        a20, d20 = G.fprop(x, w, b, gelu=True, cfg=20)
        assert torch.equal(a20, a18) and torch.equal(d20, d18)
        assert torch.equal(G.dgrad(dy, w2, cfg=20), x18)
        assert torch.equal(G.dgrad(dy, w2, cfg=20, scale=s), xs18)


@pytest.mark.parametrize("M,N,K", [(16384, 768, 3072), (16384, 2304, 768), (5000, 776, 256), (300, 200, 128)])
def test_gemm8pc_192_bit_identical(M, N, K):
    _check_192(M, N, K, 21)


@pytest.mark.parametrize("M,N,K", [(16384, 768, 3072), (16384, 2304, 768), (5000, 776, 256), (300, 200, 64)])
def test_gemm8p_192_bit_identical(M, N, K):
    """cfg 22: the one-shot 8-phase loop at 256 x 192 (one tile per block, LDS epilogue)."""
    _check_192(M, N, K, 22)


def _check_192(M, N, K, cfg):
    """cfg 21: the continuous 8-phase stream at 256 x 192 (waves of 128 x 48: one-instruction B1 region,
    7 instructions in flight, an unpaired third n-block stored 8 bytes per lane): bit-identical to the
    16x16x32 loop at the same tile (cfg 16) for bias and bias + GELU fprops; dgrad falls back to cfg 16."""
    x, w, b = _bf(M, K, seed=70), _bf(N, K, scale=0.03, seed=71), _bf(N, seed=72)
    y = G.fprop(x, w, b, cfg=cfg)
    assert rel_err(y, F.linear(x.float(), w.float(), b.float())) < 1e-2
    assert torch.equal(y, G.fprop(x, w, b, cfg=16))
    a21, d21 = G.fprop(x, w, b, gelu=True, cfg=cfg)
    a16, d16 = G.fprop(x, w, b, gelu=True, cfg=16)
    assert torch.equal(a21, a16) and torch.equal(d21, d16)
    dy, w2 = _bf(M, K, seed=73), _bf(K, N, scale=0.03, seed=74)
    assert torch.equal(G.dgrad(dy, w2, cfg=cfg), G.dgrad(dy, w2, cfg=16))
