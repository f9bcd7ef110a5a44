"""Fixed-cost vs per-K-tile cost of the bf16 GEMM on a 1x1-conv forward shape:
time over K at fixed M x N (intercept = per-tile prologue + epilogue, slope =
main loop), for igemm_k's auto policy with the LDS-staged epilogue on / off
(set_tuning(1, v)).  One JSON line per K."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from singa_amd.ops import functional as F  # noqa: E402
from singa_amd.ops import native as N  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


L = N.lib()
M = int(sys.argv[1]) if len(sys.argv) > 1 else 200704
Nn = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
for K in (64, 128, 256, 512, 1024):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(Nn, K, device="cuda").bfloat16()
    rec = {"M": M, "N": Nn, "K": K, "out_MB": M * Nn * 2 / 1e6, "in_MB": M * K * 2 / 1e6}
    for ep in (1, 0):
        L.set_tuning(1, ep)
        rec[f"us_lds{ep}"] = round(timeit(lambda: F.gemm_nt(x, w, out_dtype=torch.bfloat16)), 1)
    L.set_tuning(1, 1)
    L.set_tuning(8, 1)
    rec["us_lds1_nt"] = round(timeit(lambda: F.gemm_nt(x, w, out_dtype=torch.bfloat16)), 1)
    L.set_tuning(8, 0)
    rec["us_torch"] = round(timeit(lambda: x @ w.t()), 1)
    out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
    rec["us_fill_out"] = round(timeit(lambda: out.fill_(1.0)), 1)  # write-only pass over the output size
    print(json.dumps(rec), flush=True)
    del x, w, out
