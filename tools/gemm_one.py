"""One plain bf16 GEMM shape under one tile policy, a few launches (PMC
passes: tools/pmc_gemm.sh).  python tools/gemm_one.py --M 8192 --K 8192 --N 8192 --policy 8"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from singa_amd.ops import functional as F  # noqa: E402
from singa_amd.ops import native as N  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=8192)
ap.add_argument("--K", type=int, default=8192)
ap.add_argument("--N", type=int, default=8192)
ap.add_argument("--policy", type=int, default=0)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--f32", action="store_true", help="fp32 operands (generic kernel, ggemm.hip)")
ap.add_argument("--tile", type=int, default=0, help="fp32: ggemm_tune(0, tile)")
ap.add_argument("--splits", type=int, default=0, help="fp32: ggemm_tune(1, splits)")
ap.add_argument("--kout", action="store_true", help="fp32: B stored [K][N] (x @ W forward)")
a = ap.parse_args()
L = N.lib()
if a.f32:
    L.ggemm_tune(0, a.tile)
    L.ggemm_tune(1, a.splits)
    x = torch.randn(a.M, a.K, device="cuda")
    w = torch.randn(a.K, a.N, device="cuda") if a.kout else torch.randn(a.N, a.K, device="cuda")
    for _ in range(a.iters):
        F.matmul(x, w) if a.kout else F.gemm_nt(x, w)
else:
    x = torch.randn(a.M, a.K, device="cuda").bfloat16()
    w = torch.randn(a.N, a.K, device="cuda").bfloat16()
    L.set_tuning(4, a.policy)
    for _ in range(a.iters):
        F.gemm_nt(x, w, out_dtype=torch.bfloat16)
torch.cuda.synchronize()
print("done")
