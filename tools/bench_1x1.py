"""The ResNet-50 b1024 1x1-conv GEMM shapes (C[M][N] = A[M][K] B[N][K]^T,
bf16 out) under each existing tile policy: per shape and policy the mean
time of a launch and the compulsory-byte bandwidth (A + B + C once) -- which
kernel variant each memory-bound shape wants.

    python tools/bench_1x1.py [--iters 20] [--out profiles/r6/bench_1x1.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from singa_amd.ops import functional as F  # noqa: E402
from singa_amd.ops import native as N  # noqa: E402

SHAPES = [  # (M, N, K): stage-3 / 4 forwards and data gradients, stage-2 wide ones
    (200704, 1024, 256), (200704, 256, 1024), (802816, 512, 256), (802816, 128, 512), (50176, 2048, 512),
    (50176, 512, 2048), (200704, 1024, 512), (3211264, 128, 256), (802816, 256, 512), (200704, 512, 1024),
]
# name -> [(tuning key, value), ...]  (igemm.hip g_tune: 4 forced tile, 5 8-wave tiles, 6 single-stage cap,
# 7 early issue, 9 persistent short-K, 16 256x128 three-stage tiles)
POLICIES = {
    "default": [],
    "t256x128": [(16, 3)],
    "pingpong": [(4, 8)],
    "v2_4wave": [(5, 0)],
    "single_stage": [(6, 16)],
    "no_early_issue": [(7, 0)],
    "stream": [(18, 2)],
    "generic": [(18, 0)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--policies", default=",".join(POLICIES))
    a = ap.parse_args()
    L = N.lib()
    base = {k: L.get_tuning(k) for k in (4, 5, 6, 7, 9, 16, 18)} if hasattr(L, "get_tuning") else None
    recs = []
    for (M, Nn, K) in SHAPES:
        x = (torch.randn(M, K, device="cuda") * 0.1).bfloat16()
        w = (torch.randn(Nn, K, device="cuda") * 0.1).bfloat16()
        ref = None
        for pname in a.policies.split(","):
            for k, v in POLICIES[pname]:
                L.set_tuning(k, v)
            try:
                y = F.gemm_nt(x, w, out_dtype=torch.bfloat16)
                torch.cuda.synchronize()
                if ref is None:
                    ref = y.float()
                err = float((y.float() - ref).abs().max())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    F.gemm_nt(x, w, out_dtype=torch.bfloat16)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.iters
                gb = 2.0 * (M * K + Nn * K + M * Nn) / 1e9
                rec = {"M": M, "N": Nn, "K": K, "policy": pname, "us": round(us, 1), "TBps": round(gb * 1e3 / us, 3),
                       "TFps": round(2.0 * M * Nn * K / us * 1e-6, 1), "max_abs_diff_vs_default": err}
            finally:
                if base is not None:
                    for k, v in base.items():
                        L.set_tuning(k, v)
                else:
                    for k, v in POLICIES[pname]:
                        L.set_tuning(k, {4: 0, 5: 1, 6: 2, 7: 1, 9: 1, 16: 0, 18: 1}[k])
            recs.append(rec)
            print(json.dumps(rec), flush=True)
        del x, w, ref
    if a.out:
        with open(a.out, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
