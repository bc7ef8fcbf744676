"""Run one own-GEMM call repeatedly (for rocprofv3 --pmc passes / kernel traces).

    python tools/gemm_one.py --kind dgrad --M 16384 --N 768 --K 3072 --cfg 0 --reps 20
(kind fprop: x[M,K] w[N,K]; dgrad: dy[M,K] w[K,N]; wgrad: dy[K,M] x[K,N]; --epi gelu / geluback)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_example_amd.ops import gemm as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="dgrad")
ap.add_argument("--M", type=int, default=16384)
ap.add_argument("--N", type=int, default=768)
ap.add_argument("--K", type=int, default=3072)
ap.add_argument("--cfg", type=int, default=0)
ap.add_argument("--splits", type=int, default=1)
ap.add_argument("--epi", default="none")
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda", 0)
r = lambda *s: (torch.randn(*s, device=dev) * 0.05).to(torch.bfloat16)
if a.kind == "fprop":
    x, w, b = r(a.M, a.K), r(a.N, a.K), r(a.N)
    fn = lambda: G.fprop(x, w, b, gelu=a.epi == "gelu", cfg=a.cfg)
elif a.kind == "dgrad":
    dy, w = r(a.M, a.K), r(a.K, a.N)
    pre = r(a.M, a.N) if a.epi == "geluback" else None
    fn = lambda: G.dgrad(dy, w, dgelu=pre, cfg=a.cfg)
else:
    dy, x = r(a.K, a.M), r(a.K, a.N)
    fn = lambda: G.wgrad(dy, x, cfg=a.cfg, splits=a.splits, want_db=True)
for _ in range(a.reps):
    fn()
torch.cuda.synchronize()
print("done", a)
