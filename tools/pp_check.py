"""Correctness sweep of the ping-pong 256x256 GEMM (set_tuning(4, 8)) on
ragged shapes (M, N not tile multiples, K not a BK multiple), bf16 and fp32
outputs, against fp32 torch on the same bf16 operands."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from singa_amd.ops import functional as F  # noqa: E402
from singa_amd.ops import native as N  # noqa: E402

L = N.lib()
torch.manual_seed(0)
worst = 0.0
for (M, K, Nn) in ((1000, 200, 264), (4097, 72, 520), (300, 328, 256), (256, 64, 256), (513, 1024, 768),
                   (8, 8, 8), (2048, 4104, 1032)):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(Nn, K, device="cuda").bfloat16()  # [N][K]
    ref = x.float() @ w.float().t()
    for od in (torch.bfloat16, torch.float32):
        L.set_tuning(4, 8)
        out = F.gemm_nt(x, w, out_dtype=od).float()
        L.set_tuning(4, 0)
        base = F.gemm_nt(x, w, out_dtype=od).float()
        e = float((out - ref).norm() / ref.norm())
        eb = float((base - ref).norm() / ref.norm())
        worst = max(worst, e)
        print(f"M={M} K={K} N={Nn} {od}: rel err pp {e:.2e}  base {eb:.2e}", flush=True)
print("worst", worst)
assert worst < 5e-3
