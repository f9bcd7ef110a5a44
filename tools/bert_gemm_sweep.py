"""Tile / split-K sweep of BERT-base's projection GEMMs at the bench shape
(4096 tokens), in the orientations autograd.Linear runs them:
  fwd   y = x W          A [M][K] K-major, B = W [K][N] (K-outer), bf16 out
  dgrad dx = dy W^T       A [M][K] K-major, B = W [N][K] (K-major), bf16 out
  wgrad dW += x^T dy      A, B K-outer, fp32 atomic out (split-K)
policy = set_tuning(4, p): 0 auto, 1 128x64, 2 64x128, 3 64x64, 4 128x128,
5 128x128 8-wave.  One JSON line per (gemm, policy, splits): us, TFLOP/s.

    python tools/bert_gemm_sweep.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from singa_amd.ops import native as N

    L = N.lib()
    T = 4096
    shapes = {"qkv": (768, 2304), "proj": (768, 768), "fc1": (768, 3072), "fc2": (3072, 768)}
    g0 = torch.Generator(device="cuda").manual_seed(0)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    def timeit(fn, iters=50):
        for _ in range(5):
            fn()
        e0, e1 = ev(), ev()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3

    SPLITS = tuple(int(v) for v in os.environ.get("SWEEP_SPLITS", "0,2,4,8").split(","))
    kinds = os.environ.get("SWEEP_KINDS", "fwd,dgrad,wgrad").split(",")
    for name, (din, dout) in shapes.items():
        x = torch.randn(T, din, device="cuda", generator=g0).bfloat16()
        w = torch.randn(din, dout, device="cuda", generator=g0).bfloat16()
        dy = torch.randn(T, dout, device="cuda", generator=g0).bfloat16()
        y = torch.empty(T, dout, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(T, din, device="cuda", dtype=torch.bfloat16)
        dw = torch.zeros(din, dout, device="cuda")
        s = N.stream()
        cases = {
            # (M, N, K, call)
            "fwd": (T, dout, din, lambda sp: L.gemm(x.data_ptr(), din, 0, w.data_ptr(), dout, 1, y.data_ptr(), dout, T,
                                                    dout, din, 1.0, 0.0, 0, 0, 0, 1, 1, 0, 0, 0, s)),
            "dgrad": (T, din, dout, lambda sp: L.gemm(dy.data_ptr(), dout, 0, w.data_ptr(), dout, 0, dx.data_ptr(), din,
                                                      T, din, dout, 1.0, 0.0, 0, 0, 0, 1, 1, 0, 0, 0, s)),
            "wgrad": (din, dout, T, lambda sp: L.gemm(x.data_ptr(), din, 1, dy.data_ptr(), dout, 1, dw.data_ptr(), dout,
                                                      din, dout, T, 1.0, 1.0, 0, 0, 2, sp, 1, 0, 0, 0, s)),
        }
        for kind, (M, Nn, K, call) in cases.items():
            if kind not in kinds:
                continue
            for pol in (0, 1, 2, 3, 4, 5):
                for sp in (SPLITS if kind == "wgrad" else (1,)):
                    L.set_tuning(4, pol)
                    try:
                        us = timeit(lambda: call(sp))
                    finally:
                        L.set_tuning(4, 0)
                    print(json.dumps({"gemm": name, "kind": kind, "M": M, "N": Nn, "K": K, "policy": pol,
                                      "splits": sp, "us": round(us, 2),
                                      "TFs": round(2.0 * M * Nn * K / us * 1e-6, 1)}), flush=True)


if __name__ == "__main__":
    main()
