"""Fused attention kernel timing at BERT-base shapes (B 32, S 128, H 12,
D 64): forward, backward, and backward with the q/k/v bias-gradient column
sums (``db_acc``).

    python tools/bench_fattn.py [--iters 50]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from singa_amd.ops import functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--S", type=int, default=128)
    ap.add_argument("--H", type=int, default=12)
    a = ap.parse_args()
    B, S, H, D = a.B, a.S, a.H, 64
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(B, S, 3 * H * D, device="cuda", generator=g) * 0.5).bfloat16()
    do = torch.randn(B, S, H * D, device="cuda", generator=g).bfloat16()
    mask = torch.zeros(B, 1, 1, S, device="cuda")
    scale = 1.0 / math.sqrt(D)
    o, st = F.attention_qkv_fwd(qkv, H, mask, scale)
    db = torch.zeros(3 * H * D, device="cuda")

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) * 1e3 / a.iters, 2)

    rec = {"B": B, "S": S, "H": H,
           "fwd_us": timed(lambda: F.attention_qkv_fwd(qkv, H, mask, scale)),
           "bwd_us": timed(lambda: F.attention_qkv_bwd(qkv, st, do, H, scale)),
           "bwd_dbias_us": timed(lambda: F.attention_qkv_bwd(qkv, st, do, H, scale, db_acc=db))}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
