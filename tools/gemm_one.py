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
a = ap.parse_args()
L = N.lib()
x = torch.randn(a.M, a.K, device="cuda").bfloat16()
w = torch.randn(a.N, a.K, device="cuda").bfloat16()
L.set_tuning(4, a.policy)
for _ in range(a.iters):
    F.gemm_nt(x, w, out_dtype=torch.bfloat16)
torch.cuda.synchronize()
print("done")
