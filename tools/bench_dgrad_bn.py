"""Microbenchmark: accumulate-dgrad of a 1x1 conv into a residual BN(+ReLU)
output gradient, with and without the BN-backward partial sums fused into
its epilogue (stats_mode 2, 1-bit mask), vs the separate reduction pass."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from singa_amd.ops import functional as F  # noqa: E402
from singa_amd.ops import native as N  # noqa: E402


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda")
    L = N.lib()
    for (C, K, H) in ((256, 64, 56), (512, 128, 28), (1024, 256, 14), (2048, 512, 7)):
        B = a.batch
        cl = torch.channels_last
        x = torch.randn(B, C, H, H, device=dev).bfloat16().contiguous(memory_format=cl)   # BN input z3
        dy = torch.randn(B, K, H, H, device=dev).bfloat16().contiguous(memory_format=cl)  # conv1 output grad
        w = (torch.randn(K, C, 1, 1, device=dev) * 0.05).bfloat16().contiguous(memory_format=cl)
        acc = torch.randn(B, C, H, H, device=dev).bfloat16().contiguous(memory_format=cl)
        gam, bet = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
        y, st = F.batchnorm_fwd(x, gam, bet, torch.zeros(C, device=dev), torch.ones(C, device=dev), True, relu=True,
                                residual=acc, want_mask=True)
        wt = torch.empty(K * C, dtype=torch.bfloat16, device=dev)
        ws = torch.zeros(32 * 2 * C, device=dev)
        R = B * H * H
        t_acc = timeit(lambda: L.conv_dgrad_acc(dy.data_ptr(), w.data_ptr(), acc.data_ptr(), B, H, H, C, K, 1, 1, H, H,
                                                1, 1, 0, 0, 1, 1, 0, 1.0, N.stream(), wt.data_ptr()))
        t_fused = timeit(lambda: L.conv_dgrad_bn(dy.data_ptr(), w.data_ptr(), acc.data_ptr(), B, H, H, C, K, 1, 1, H,
                                                 H, 1, 1, 0, 0, 1, 1, wt.data_ptr(), ws.data_ptr(), x.data_ptr(),
                                                 st.mean.data_ptr(), st.invstd.data_ptr(), st.scale.data_ptr(),
                                                 st.shift.data_ptr(), N.stream(), 1.0, st.mask.data_ptr()))
        def bwd(with_ws):
            g = acc
            if with_ws:
                g._sg_bnbwd_ws = (ws, 32)
            elif hasattr(g, "_sg_bnbwd_ws"):
                del g._sg_bnbwd_ws
            F.batchnorm_bwd(x, g, gam, st, None, need_dres=True, relu=True)
        t_bn_full = timeit(lambda: bwd(False))
        t_bn_ws = timeit(lambda: bwd(True))
        print(json.dumps({"C": C, "K": K, "H": H, "R": R, "dgrad_acc_ms": round(t_acc, 3),
                          "dgrad_acc_bn_ms": round(t_fused, 3), "bn_bwd_full_ms": round(t_bn_full, 3),
                          "bn_bwd_from_ws_ms": round(t_bn_ws, 3)}), flush=True)


if __name__ == "__main__":
    main()
