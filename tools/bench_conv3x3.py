"""Time the ResNet-50 stage-1 3x3 convolution (N x 56 x 56 x 64 -> 64, bf16,
stride 1, pad 1) forward (with fused BN statistics) and data gradient (with
the identity-sum masked gradient sum) on the persistent kernel
(csrc/kernels/conv3x3.hip) and on the generic implicit GEMM
(``conv3x3_set(0)``).  One JSON line per (pass, path).

  python tools/bench_conv3x3.py [--batch 1024] [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from singa_amd.ops import native as N  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None, help="fwd | dgrad: run that pass on the persistent kernel --iters times "
                    "with no timing (for rocprofv3 counter passes)")
    a = ap.parse_args()
    L = N.lib()
    dev = torch.device("cuda", 0)
    n, h = a.batch, 56
    x = torch.randn(n, h, 56, 64, device=dev).bfloat16()
    w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).bfloat16()
    y = torch.empty_like(x)
    ws = torch.zeros(32 * 2 * 64, dtype=torch.float32, device=dev)
    wt = torch.empty(64 * 64 * 9, dtype=torch.bfloat16, device=dev)
    mask = torch.randint(0, 256, (n * h * 56 * 8,), dtype=torch.uint8, device=dev)
    s = N.stream()
    flops = 2.0 * n * h * 56 * 64 * 64 * 9
    nbytes = 2.0 * 2 * n * h * 56 * 64

    def fwd():
        L.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, n, h, 56, 64, 64, 3, 3, h, 56, 1, 1, 1, 1, 1, 1, 0, 0,
                   s, ws.data_ptr())

    def fwd_nostats():
        L.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, n, h, 56, 64, 64, 3, 3, h, 56, 1, 1, 1, 1, 1, 1, 0, 0,
                   s, 0)

    def dgrad():
        L.conv_dgrad_bn(x.data_ptr(), w.data_ptr(), y.data_ptr(), n, h, 56, 64, 64, 3, 3, h, 56, 1, 1, 1, 1, 1, 1,
                        wt.data_ptr(), ws.data_ptr(), 0, 0, 0, 0, 0, s, 0.0, mask.data_ptr())

    if a.only:
        fn = fwd if a.only == "fwd" else dgrad
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        return
    paths = (1,) if os.environ.get("SG_C3_DBG") else (1, 0)
    for name, fn in (("fwd+stats", fwd), ("fwd", fwd_nostats), ("dgrad+masksum", dgrad)):
        for on in paths:
            L.conv3x3_set(on)
            ms = timeit(fn, a.iters)
            print(json.dumps({"pass": name, "path": "persistent" if on else "generic", "batch": n, "ms": round(ms, 4),
                              "tflops": round(flops / ms / 1e9, 1), "tb_s": round(nbytes / ms / 1e9, 2)}), flush=True)
    L.conv3x3_set(1)


if __name__ == "__main__":
    main()
