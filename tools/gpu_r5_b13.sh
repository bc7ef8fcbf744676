#!/bin/bash
# Round-5 batch 13: attention dK/dV with both query halves' S / dP issued ahead of the softmax
# gradient (variant 13 = 5 | 8) vs the default (5): bit equality of dQ / dK / dV, then timings.
set -o pipefail
O=gpurun_out/${1:-r5_b13}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python - > $O/equal.txt 2>&1 <<'PY' || { cat $O/equal.txt; exit 1; }
import math, torch
from pytorch_distributed_example_amd._ext import kernels
K = kernels()
B, T, H, D = 4, 1024, 12, 64
C = H * D
torch.manual_seed(0)
qkv = torch.randn(B, T, 3 * C, device="cuda").to(torch.bfloat16)
q, k, v = qkv[:, :, :C], qkv[:, :, C:2 * C], qkv[:, :, 2 * C:]
o = torch.empty(B, T, C, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B * H * T, device="cuda")
do = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
outs = []
for var in (5, 13):
    K.attn_set_variant(var)
    dqkv = torch.empty_like(qkv)
    Dd = torch.empty(B * H * T, device="cuda")
    K.attn_fwd(q, k, v, o, lse, H, 1 / math.sqrt(D))
    K.attn_bwd(q, k, v, o, do, lse, Dd, dqkv[:, :, :C], dqkv[:, :, C:2 * C], dqkv[:, :, 2 * C:], H, 1 / math.sqrt(D))
    torch.cuda.synchronize()
    outs.append(dqkv.clone())
K.attn_set_variant(5)
print("bit-identical:", torch.equal(outs[0], outs[1]), "max diff", (outs[0].float() - outs[1].float()).abs().max().item())
assert torch.equal(outs[0], outs[1])
PY
cat $O/equal.txt
timeout -k 10 200 python tools/attn_bench.py --variants 5,13,5,13,5,13 > $O/bench.jsonl 2> $O/bench.err || exit 1
cat $O/bench.jsonl
