"""Plain-GEMM microbenchmark on the BERT-base projection shapes (tokens =
batch * seq): the MFMA kernel's forward (x @ W + bias), data-gradient
(dy @ W^T) and weight-gradient (x^T @ dy, fp32 split-K accumulate) calls
under each tile policy (``set_tuning(4, v)``: 0 auto, 1 128x64, 2 64x128,
3 64x64, 4 128x128, 5 8-wave 128x128), against torch.matmul (hipBLASLt) on
the same bf16 operands.  One JSON line per (shape, kind)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from singa_amd.ops import functional as F  # noqa: E402
from singa_amd.ops import native as N  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--policies", default="0,1,2,3,4,5")
    a = ap.parse_args()
    L = N.lib()
    dev = torch.device("cuda", 0)
    M = a.tokens
    for (K, Nn) in ((768, 2304), (768, 768), (768, 3072), (3072, 768)):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = torch.randn(K, Nn, device=dev).bfloat16()
        dy = torch.randn(M, Nn, device=dev).bfloat16()
        bias = torch.randn(Nn, device=dev)
        gw = torch.zeros(K, Nn, device=dev)
        wt = w.t().contiguous()
        flops = 2.0 * M * K * Nn
        kinds = {
            "fwd": (lambda: F.matmul(x, w, out_dtype=torch.bfloat16, bias=bias), lambda: torch.addmm(bias.bfloat16(), x, w)),
            "dgrad": (lambda: F.gemm_nt(dy, w, out_dtype=torch.bfloat16), lambda: dy @ wt),
            "wgrad": (lambda: F.gemm_tn_acc(x, dy, gw), lambda: x.t() @ dy),
        }
        for kind, (ours, ref) in kinds.items():
            rec = {"M": M, "K": K, "N": Nn, "kind": kind}
            for pol in [int(v) for v in a.policies.split(",")]:
                L.set_tuning(4, pol)
                rec[f"us_p{pol}"] = round(timeit(ours), 1)
            L.set_tuning(4, 0)
            rec["us_torch"] = round(timeit(ref), 1)
            best = min(v for k, v in rec.items() if k.startswith("us_p"))
            rec["TF_best_ours"] = round(flops / best / 1e6, 1)
            rec["TF_torch"] = round(flops / rec["us_torch"] / 1e6, 1)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
