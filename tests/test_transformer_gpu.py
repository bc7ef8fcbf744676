"""Transformer kernels (bf16) vs plain PyTorch fp32 references of the same ops, and GPT-2 model /
optimizer parity (GPU bf16 vs CPU fp32 with identical weights)."""
import math

import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_example_amd.ops import transformer as T
from pytorch_distributed_example_amd.models import GPTConfig, build_gpt2
from pytorch_distributed_example_amd.optim import AdamWMaster

pytestmark = pytest.mark.gpu
dev = "cuda"


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


@pytest.mark.parametrize("N,C", [(300, 768), (64, 1000), (5, 128), (17, 2048)])
def test_layernorm(N, C):
    torch.manual_seed(0)
    x = (torch.randn(N, C) * 2 + 0.5).to(dev, torch.bfloat16).requires_grad_()
    w = (1 + 0.1 * torch.randn(C)).to(dev, torch.bfloat16).requires_grad_()
    b = (0.1 * torch.randn(C)).to(dev, torch.bfloat16).requires_grad_()
    y = T.layer_norm(x, w, b)
    g = torch.randn(N, C).to(dev, torch.bfloat16)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = F.layer_norm(xr, (C,), wr, br, 1e-5)
    yr.backward(g.float())
    assert rel_err(y, yr) < 1e-2
    assert rel_err(x.grad, xr.grad) < 2e-2
    assert rel_err(w.grad, wr.grad) < 2e-2
    assert rel_err(b.grad, br.grad) < 2e-2


def test_gelu():
    torch.manual_seed(1)
    x = (torch.randn(4096) * 3).to(dev, torch.bfloat16).requires_grad_()
    y = T.gelu(x)
    g = torch.randn(4096).to(dev, torch.bfloat16)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    yr = F.gelu(xr, approximate="tanh")
    yr.backward(g.float())
    assert rel_err(y, yr) < 1e-2
    assert rel_err(x.grad, xr.grad) < 2e-2


@pytest.mark.parametrize("N,V,Vp", [(37, 1000, 1024), (8, 50257, 50304)])
def test_lm_head_loss(N, V, Vp):
    torch.manual_seed(2)
    C = 64
    h = torch.randn(N, C).to(dev, torch.bfloat16).requires_grad_()
    w = (0.5 * torch.randn(Vp, C)).to(dev, torch.bfloat16).requires_grad_()
    tgt = torch.randint(0, V, (N,), device=dev)
    loss = T.lm_head_loss(h, w, tgt, V)
    loss.backward()
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    lr = F.cross_entropy((hr @ wr.t())[:, :V], tgt)
    lr.backward()
    assert abs(loss.item() - lr.item()) < 2e-2 * max(1.0, abs(lr.item()))
    assert rel_err(h.grad, hr.grad) < 3e-2
    assert rel_err(w.grad, wr.grad) < 3e-2
    assert w.grad[V:].abs().max().item() == 0.0        # padded vocab rows get no gradient


def test_embedding():
    torch.manual_seed(3)
    B, Tn, C, Vp = 4, 128, 128, 512
    idx = torch.randint(0, 40, (B, Tn), device=dev)   # many repeats -> exercises the atomic path
    wte = torch.randn(Vp, C).to(dev, torch.bfloat16).requires_grad_()
    wpe = torch.randn(Tn, C).to(dev, torch.bfloat16).requires_grad_()
    x = T.embedding(idx, wte, wpe)
    g = torch.randn(B, Tn, C).to(dev, torch.bfloat16)
    x.backward(g)
    wter, wper = wte.detach().float().requires_grad_(), wpe.detach().float().requires_grad_()
    xr = F.embedding(idx, wter) + wper.unsqueeze(0)
    xr.backward(g.float())
    assert rel_err(x, xr) < 1e-2
    assert rel_err(wte.grad, wter.grad) < 2e-2
    assert rel_err(wpe.grad, wper.grad) < 2e-2
    # scratch is left clean: a second backward gives the same result
    wte.grad = None
    T.embedding(idx, wte, wpe).backward(g)
    assert rel_err(wte.grad, wter.grad) < 2e-2


def _attn_ref(qkv, H):
    B, Tn, C3 = qkv.shape
    C = C3 // 3
    q, k, v = qkv.float().split(C, dim=2)
    q, k, v = (t.reshape(B, Tn, H, C // H).transpose(1, 2) for t in (q, k, v))
    s = (q @ k.transpose(-1, -2)) / math.sqrt(C // H)
    mask = torch.triu(torch.ones(Tn, Tn, dtype=torch.bool, device=qkv.device), 1)
    s = s.masked_fill(mask, float("-inf"))
    y = torch.softmax(s, -1) @ v
    return y.transpose(1, 2).reshape(B, Tn, C)


@pytest.mark.parametrize("B,Tn,H", [(2, 256, 3), (1, 128, 1), (1, 1024, 12), (3, 512, 5)])
def test_flash_attention(B, Tn, H):
    torch.manual_seed(4)
    C = 64 * H
    qkv = torch.randn(B, Tn, 3 * C).to(dev, torch.bfloat16).requires_grad_()
    y = T.causal_attention(qkv, H)
    g = torch.randn(B, Tn, C).to(dev, torch.bfloat16)
    y.backward(g)
    qr = qkv.detach().float().requires_grad_()
    yr = _attn_ref(qr, H)
    yr.backward(g.float())
    assert rel_err(y, yr) < 2e-2
    dq, dk, dv = qkv.grad.split(C, dim=2)
    rq, rk, rv = qr.grad.split(C, dim=2)
    assert rel_err(dv, rv) < 3e-2
    assert rel_err(dk, rk) < 3e-2
    assert rel_err(dq, rq) < 3e-2


def test_flash_attention_block_maps_agree():
    """The XCD-grouped block map (any group size, partial last group) computes exactly what the
    plain block order computes: every block's work is the same, only its placement changes."""
    from pytorch_distributed_example_amd._ext import kernels
    K = kernels()
    torch.manual_seed(6)
    B, Tn, H = 3, 384, 7
    C = 64 * H
    qkv = torch.randn(B, Tn, 3 * C).to(dev, torch.bfloat16)
    g = torch.randn(B, Tn, C).to(dev, torch.bfloat16)
    outs = []
    try:
        for grp in (255, 0, 3, 16):
            K.attn_set_variant(5 | (grp << 8))
            x = qkv.clone().requires_grad_()
            y = T.causal_attention(x, H)
            y.backward(g)
            outs.append((y.detach(), x.grad))
    finally:
        K.attn_set_variant(5)
    for y, dx in outs[1:]:
        assert torch.equal(y, outs[0][0]) and torch.equal(dx, outs[0][1])


def _tiny_cfg():
    return GPTConfig(block_size=128, vocab_size=1000, padded_vocab=1024, n_layer=2, n_head=2, n_embd=128)


def _gpt2_parity(break_layer: bool = False):
    """GPT-2 (4 layers, d 128, T 128, B 4) bf16 GPU vs an fp32 CPU twin with identical bf16-representable
    weights: the residual stream after every block (cosine >= 0.995 and relative L2 error), the
    loss, and every parameter gradient (cosine >= 0.99).  Returns the list of failures."""
    from pytorch_distributed_example_amd.ops import transformer as T
    cfg = GPTConfig(block_size=128, vocab_size=1000, padded_vocab=1024, n_layer=4, n_head=2, n_embd=128)
    g = build_gpt2(cfg, seed=0, device=dev)
    c = build_gpt2(cfg, seed=0, dtype=torch.float32)
    with torch.no_grad():
        for pc, pg in zip(c.parameters(), g.parameters()):
            pc.copy_(pg.float())          # identical (bf16-representable) weights
        if break_layer:                   # deliberately broken: block 1's ln_1 weight and bias swapped
            ln = g.transformer.h[1].ln_1
            w = ln.weight.detach().clone()
            ln.weight.copy_(ln.bias)
            ln.bias.copy_(w)
    torch.manual_seed(5)
    idx = torch.randint(0, cfg.vocab_size, (4, 128))
    tgt = torch.randint(0, cfg.vocab_size, (4, 128))

    def streams(m, i):
        t = m.transformer
        x = T.embedding(i, t.wte.weight, t.wpe.weight)
        delta, out = None, []
        for blk in t.h:
            x, delta = blk.forward_deferred(x, delta)
            out.append((x.float() + (delta.float() if delta is not None else 0)).detach())
        return out

    with torch.no_grad():
        sg, sc = streams(g, idx.to(dev)), streams(c, idx)
    fails = []
    for k, (a, b) in enumerate(zip(sg, sc)):
        cs = F.cosine_similarity(a.double().flatten().cpu(), b.double().flatten(), dim=0).item()
        e = ((a.double().cpu() - b.double()).norm() / b.double().norm()).item()
        if not (cs >= 0.995 and e < 3e-2):
            fails.append(f"block {k} residual stream: cos {cs:.5f}, rel L2 err {e:.3e}")
    lg = g(idx.to(dev), tgt.to(dev))
    lc = c(idx, tgt)
    lg.backward()
    lc.backward()
    if not abs(lg.item() - lc.item()) < 1e-2:
        fails.append(f"loss {lg.item():.5f} vs {lc.item():.5f}")
    for (n, pg), pc in zip(g.named_parameters(), c.parameters()):
        cos = F.cosine_similarity(pg.grad.float().flatten().cpu(), pc.grad.flatten(), dim=0).item()
        if not cos >= 0.99:
            fails.append(f"grad {n}: cos {cos:.4f}")
    return fails


def test_gpt2_gpu_matches_cpu_fp32():
    """Verdict r3 next 6: whole-model parity with per-layer residual-stream checks."""
    fails = _gpt2_parity()
    assert not fails, fails


def test_gpt2_parity_catches_broken_layer():
    fails = _gpt2_parity(break_layer=True)
    assert fails, "a swapped LayerNorm weight/bias in one block went unnoticed"
    assert any("block 1" in f for f in fails), fails


def test_adamw_master_matches_torch():
    torch.manual_seed(6)
    p16 = [torch.randn(64, 33).to(dev, torch.bfloat16).requires_grad_(), torch.randn(100).to(dev, torch.bfloat16)
           .requires_grad_()]
    ref = [p.detach().float().clone().requires_grad_() for p in p16]
    opt = AdamWMaster([{"params": [p16[0]], "weight_decay": 0.1}, {"params": [p16[1]], "weight_decay": 0.0}],
                      lr=1e-2, betas=(0.9, 0.95))
    ropt = torch.optim.AdamW([{"params": [ref[0]], "weight_decay": 0.1}, {"params": [ref[1]], "weight_decay": 0.0}],
                             lr=1e-2, betas=(0.9, 0.95), foreach=False)
    for _ in range(4):
        grads = [torch.randn_like(r) for r in ref]
        for p, r, gg in zip(p16, ref, grads):
            p.grad = gg.to(torch.bfloat16)
            r.grad = p.grad.float()
        opt.step()
        ropt.step()
    for p, r in zip(p16, ref):
        st = opt.state[p]
        assert torch.allclose(st["master"], r.detach(), atol=1e-5, rtol=1e-4)
        assert rel_err(p, r) < 1e-2


def test_adamw_master_clipping():
    torch.manual_seed(7)
    p = torch.randn(256).to(dev, torch.bfloat16).requires_grad_()
    r = p.detach().float().clone().requires_grad_()
    opt = AdamWMaster([p], lr=1e-2, weight_decay=0.0, max_grad_norm=0.5)
    ropt = torch.optim.AdamW([r], lr=1e-2, weight_decay=0.0, betas=(0.9, 0.95), foreach=False)
    g = torch.randn(256) * 3
    p.grad = g.to(dev, torch.bfloat16)
    r.grad = p.grad.float()
    torch.nn.utils.clip_grad_norm_([r], 0.5)
    opt.step()
    ropt.step()
    assert torch.allclose(opt.state[p]["master"], r.detach(), atol=1e-5, rtol=1e-4)


def test_gpt2_trains():
    cfg = _tiny_cfg()
    m = build_gpt2(cfg, seed=1, device=dev)
    opt = AdamWMaster(m.decay_groups(0.1), lr=3e-3, max_grad_norm=1.0)
    torch.manual_seed(8)
    idx = torch.randint(0, cfg.vocab_size, (4, 128), device=dev)
    losses = []
    for _ in range(30):
        opt.zero_grad()
        loss = m(idx, torch.roll(idx, -1, 1))
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0], losses


def test_gpt2_step_replays_as_hipgraph():
    """The bench's whole-step hipGraph (capturable AdamW: device step count): replays of the captured
    step give the same weights as the same number of eager steps (bias corrections included)."""
    cfg = _tiny_cfg()
    torch.manual_seed(9)
    batches = [torch.randint(0, cfg.vocab_size, (2, 129), device=dev) for _ in range(5)]

    def run(graph_mode):
        m = build_gpt2(cfg, seed=2, device=dev)
        opt = AdamWMaster(m.decay_groups(0.1), lr=3e-3, max_grad_norm=1.0, capturable=graph_mode)

        def one(b):
            opt.zero_grad()
            loss = m(b[:, :-1], b[:, 1:])
            loss.backward()
            opt.step()
            return loss.detach()

        losses = [one(batches[0]).item(), one(batches[1]).item()]      # two eager steps first (warm-up)
        if not graph_mode:
            losses += [one(b).item() for b in batches[2:]]
        else:
            sb = batches[2].clone()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                sl = one(sb)
            for b in batches[2:]:
                sb.copy_(b)
                g.replay()
                losses.append(sl.item())
        torch.cuda.synchronize()
        return losses, [p.detach().float().clone() for p in m.parameters()], opt

    le, pe, _ = run(False)
    lg, pg, opt = run(True)
    # (the embedding backward accumulates with float atomics: equal up to summation order)
    assert le == pytest.approx(lg, rel=2e-3)
    for a, b in zip(pe, pg):
        assert rel_err(a, b) < 1e-2
    assert float(next(iter(opt.state.values()))["step"]) == 5.0


@pytest.mark.parametrize("N,fin,fout", [(16384, 768, 2304), (4096, 3072, 768), (300, 64, 1000), (37, 128, 24)])
def test_linear_splitk_and_bias_grad(N, fin, fout):
    torch.manual_seed(10)
    x = torch.randn(N, fin).to(dev, torch.bfloat16).requires_grad_()
    w = (torch.randn(fout, fin) / fin ** 0.5).to(dev, torch.bfloat16).requires_grad_()
    b = torch.randn(fout).to(dev, torch.bfloat16).requires_grad_()
    y = T.linear(x, w, b)
    g = torch.randn(N, fout).to(dev, torch.bfloat16)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = F.linear(xr, wr, br)
    yr.backward(g.float())
    assert rel_err(y, yr) < 1e-2
    assert rel_err(x.grad, xr.grad) < 2e-2
    assert rel_err(w.grad, wr.grad) < 2e-2
    assert rel_err(b.grad, br.grad) < 2e-2


def test_linear_rejects_unsupported_shapes():
    """No silent library fallback: in_features % 64 != 0 raises on GPU."""
    x = torch.randn(8, 40, device=dev, dtype=torch.bfloat16)
    w = torch.randn(24, 40, device=dev, dtype=torch.bfloat16)
    with pytest.raises(NotImplementedError):
        T.linear(x, w, None)


def test_mlp_fused_matches_fp32():
    """MLP as one op (c_fc + bias + GELU epilogue, GELU backward in c_proj's dgrad epilogue)."""
    torch.manual_seed(11)
    N, C = 1000, 256
    x = torch.randn(N, C).to(dev, torch.bfloat16).requires_grad_()
    ps = [(torch.randn(4 * C, C) / C ** 0.5), 0.1 * torch.randn(4 * C), (torch.randn(C, 4 * C) / (4 * C) ** 0.5),
          0.1 * torch.randn(C)]
    ps = [p.to(dev, torch.bfloat16).requires_grad_() for p in ps]
    y = T.mlp(x, *ps)
    g = torch.randn(N, C).to(dev, torch.bfloat16)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    pr = [p.detach().float().requires_grad_() for p in ps]
    yr = F.linear(F.gelu(F.linear(xr, pr[0], pr[1]), approximate="tanh"), pr[2], pr[3])
    yr.backward(g.float())
    assert rel_err(y, yr) < 2e-2
    assert rel_err(x.grad, xr.grad) < 3e-2
    for p, q in zip(ps, pr):
        assert rel_err(p.grad, q.grad) < 3e-2


def test_layer_norm_residual_fused_grad():
    """(x, LN(x)) with the residual gradient folded into the LN backward kernel vs fp32 autograd."""
    from pytorch_distributed_example_amd.ops.transformer import layer_norm_residual
    torch.manual_seed(21)
    x = torch.randn(96, 384).to("cuda", torch.bfloat16).requires_grad_()
    w = (1 + 0.1 * torch.randn(384)).to("cuda", torch.bfloat16).requires_grad_()
    b = (0.1 * torch.randn(384)).to("cuda", torch.bfloat16).requires_grad_()
    g1 = torch.randn(96, 384, device="cuda")
    g2 = torch.randn(96, 384, device="cuda")
    xr, y = layer_norm_residual(x, w, b)
    ((xr.float() * g1).sum() + (y.float() * g2).sum()).backward()
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    yf = torch.nn.functional.layer_norm(xf, (384,), wf, bf, 1e-5)
    ((xf * g1).sum() + (yf * g2).sum()).backward()
    for a, r in ((x.grad, xf.grad), (w.grad, wf.grad), (b.grad, bf.grad)):
        err = ((a.float() - r).abs().max() / r.abs().max()).item()
        assert err < 2e-2, err


@pytest.mark.parametrize("N,C", [(96, 384), (16384, 768), (7, 2048)])
def test_add_layer_norm_residual_fused(N, C):
    """(x + d, LN(x + d)) with the residual add inside the LN kernel: the stored sum is exactly the
    bf16 add, LN and all gradients match an fp32 reference (x and d get the same gradient)."""
    from pytorch_distributed_example_amd.ops.transformer import add_layer_norm_residual
    torch.manual_seed(22)
    x = torch.randn(N, C).to(dev, torch.bfloat16).requires_grad_()
    d = (0.5 * torch.randn(N, C)).to(dev, torch.bfloat16).requires_grad_()
    w = (1 + 0.1 * torch.randn(C)).to(dev, torch.bfloat16).requires_grad_()
    b = (0.1 * torch.randn(C)).to(dev, torch.bfloat16).requires_grad_()
    g1 = torch.randn(N, C, device=dev)
    g2 = torch.randn(N, C, device=dev)
    s, y = add_layer_norm_residual(x, d, w, b)
    assert torch.equal(s, x.detach() + d.detach())
    ((s.float() * g1).sum() + (y.float() * g2).sum()).backward()
    xf, df, wf, bf = (t.detach().float().requires_grad_() for t in (x, d, w, b))
    sf = xf + df
    yf = F.layer_norm(sf, (C,), wf, bf, 1e-5)
    ((sf * g1).sum() + (yf * g2).sum()).backward()
    assert rel_err(y, yf) < 1e-2
    for a, r in ((x.grad, xf.grad), (d.grad, df.grad), (w.grad, wf.grad), (b.grad, bf.grad)):
        assert rel_err(a, r) < 2e-2


@pytest.mark.parametrize("case", ["shape", "dtype"])
def test_add_layer_norm_residual_unsupported_raises(case):
    """Verdict r3 weak 6: mismatched residual operands raise on GPU instead of running ATen."""
    from pytorch_distributed_example_amd.ops.transformer import add_layer_norm_residual
    x = torch.randn(8, 768, device=dev, dtype=torch.bfloat16)
    d = torch.randn(4, 768, device=dev, dtype=torch.bfloat16) if case == "shape" else x.float()
    w = torch.ones(768, device=dev, dtype=torch.bfloat16)
    with pytest.raises(NotImplementedError):
        add_layer_norm_residual(x, d, w, torch.zeros_like(w))


@pytest.mark.parametrize("variant", ["1", "2"])
def test_xent_kernel_matches_torch(variant, monkeypatch):
    """Fused softmax-CE over the padded GPT-2 vocab (the register-resident kernels: PDE_XENT_V=1 the
    online-softmax one, 2 = default the single-exp one with the padding pre-filled to -inf): per-row
    loss and the in-place dlogits vs fp32 torch, incl. a target in the last (masked) chunk, target 0
    and an ignored row (-1); padding columns get zero gradient."""
    from pytorch_distributed_example_amd._ext import kernels
    monkeypatch.setenv("PDE_XENT_V", variant)
    torch.manual_seed(11)
    N, V, Vp = 64, 50257, 50304
    logits = (3 * torch.randn(N, Vp)).to(dev, torch.bfloat16)
    tg = torch.randint(0, V, (N,), device=dev)
    tg[0], tg[1], tg[2] = V - 1, 0, -1
    ref = logits.float()[:, :V]
    rows = torch.empty(N, device=dev)
    scale = 1.0 / N
    L = logits.clone()
    kernels().xent_bf16(L, tg, V, scale, rows, True)
    valid = tg >= 0
    lse = torch.logsumexp(ref, 1)
    want_loss = torch.where(valid, lse - ref.gather(1, tg.clamp_min(0)[:, None])[:, 0], torch.zeros_like(lse))
    assert (rows - want_loss).abs().max().item() < 2e-3
    g = torch.softmax(ref, 1)
    g[torch.arange(N, device=dev)[valid], tg[valid]] -= 1
    g = g * scale * valid[:, None].float()
    got = L.float()
    assert rel_err(got[:, :V], g) < 1e-2
    assert got[:, V:].abs().max().item() == 0.0
    assert got[2].abs().max().item() == 0.0                # ignored row


@pytest.mark.parametrize("variant", ["1", "2"])
def test_xent_small_probabilities_elementwise(variant, monkeypatch):
    """softmax-CE gradients of tiny probabilities (a near-uniform row, p ~ 2e-5 over the
    GPT-2 vocab, and rows with one dominant logit, p ~ 1e-6 elsewhere) match fp32 torch ELEMENTWISE on
    the non-target columns -- below fp16's normal range the single-exp kernel's packed probabilities
    would lose their precision (the kernel keeps 2^15 p)."""
    from pytorch_distributed_example_amd._ext import kernels
    monkeypatch.setenv("PDE_XENT_V", variant)
    torch.manual_seed(13)
    N, V, Vp = 16, 50257, 50304
    logits = 0.01 * torch.randn(N, Vp)
    logits[8:, 7] = 14.0                                   # rows 8..15: dominant logit, tails ~ 8e-7
    logits = logits.to(dev, torch.bfloat16)
    tg = torch.randint(0, V, (N,), device=dev)
    ref = logits.float()[:, :V]
    rows = torch.empty(N, device=dev)
    L = logits.clone()
    kernels().xent_bf16(L, tg, V, 1.0, rows, True)
    g = torch.softmax(ref, 1)
    g[torch.arange(N, device=dev), tg] -= 1
    got = L.float()[:, :V]
    mask = torch.ones_like(g, dtype=torch.bool)
    mask[torch.arange(N, device=dev), tg] = False
    rel = ((got - g).abs() / g.abs().clamp_min(1e-30))[mask]
    assert rel.max().item() < 1.6e-2, rel.max().item()      # bf16 output rounding (2^-8) plus fp32 math
    lse = torch.logsumexp(ref, 1)
    assert (rows - (lse - ref.gather(1, tg[:, None])[:, 0])).abs().max().item() < 2e-3


def test_scale_bf16_matches_torch():
    """In-place bf16 scale by a device scalar (LM-head dgrad loss-gradient scale): matches the fp32
    product rounded once to bf16, over a grid-stride tail (n8 not a multiple of the block)."""
    from pytorch_distributed_example_amd._ext import kernels
    torch.manual_seed(12)
    x = torch.randn(1000 * 8 + 8 * 37, device=dev).to(torch.bfloat16)
    s = torch.tensor([0.3712], device=dev)
    want = (x.float() * s).to(torch.bfloat16)
    kernels().scale_bf16(x, s)
    assert torch.equal(x, want)
