"""Ceiling probe for the bf16 MFMA GEMM core: plain bf16 GEMMs of the
ResNet-50 1x1-conv forward shapes (pixels x Cin -> Cout at b1024) and a large
square, our kernel under each tile policy (``set_tuning(4, v)``: 0 auto,
5 8-wave 128x128, 6 8-wave 256x64 4-stage, 7 8-wave 256x128 3-stage) against
torch.matmul (hipBLASLt) on the same operands.  One JSON line per shape."""
import argparse
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
    return e0.elapsed_time(e1) / iters * 1e3  # us


SHAPES = [  # (M, K, N)
    (8192, 8192, 8192),
    (200704, 256, 1024),   # layer3 expand
    (200704, 1024, 256),   # layer3 reduce
    (50176, 512, 2048),    # layer4 expand
    (50176, 2048, 512),    # layer4 reduce
    (802816, 512, 128),    # layer2 reduce
    (802816, 128, 512),    # layer2 expand
    (3211264, 64, 256),    # layer1 expand
    (200704, 2304, 256),   # layer3 3x3 as a dense GEMM (K = 9*256)
    (50176, 4608, 512),    # layer4 3x3 as a dense GEMM
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--policies", default="0,5,7")
    a = ap.parse_args()
    L = N.lib()
    dev = torch.device("cuda", 0)
    for (M, K, Nn) in SHAPES:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = torch.randn(Nn, K, device=dev).bfloat16()  # [N][K]: both operands K-major (the 1x1-conv forward layout)
        flops = 2.0 * M * K * Nn
        byts = 2.0 * (M * K + K * Nn + M * Nn)
        rec = {"M": M, "K": K, "N": Nn}
        ref = None
        if M * Nn <= 300_000_000:
            ref = (x[:4096].float() @ w.float().t())
        for pol in [int(v) for v in a.policies.split(",")]:
            L.set_tuning(4, pol)
            us = timeit(lambda: F.gemm_nt(x, w, out_dtype=torch.bfloat16))
            rec[f"TF_p{pol}"] = round(flops / us / 1e6, 1)
            if ref is not None:
                out = F.gemm_nt(x, w, out_dtype=torch.bfloat16)[:4096].float()
                rec[f"err_p{pol}"] = float((out - ref).norm() / ref.norm())
        L.set_tuning(4, 0)
        us = timeit(lambda: x @ w.t())
        rec["TF_torch"] = round(flops / us / 1e6, 1)
        rec["roof_us"] = round(max(flops / 2.5e15, byts / 6.5e12) * 1e6, 1)
        print(json.dumps(rec), flush=True)
        del x, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
