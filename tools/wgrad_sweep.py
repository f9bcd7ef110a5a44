"""Split-count sweep of the 8-wave split-K conv weight gradient on ResNet-50's
b1024 shapes (knob 12 forces the split count; 0 = the policy's choice, knob 13
selects the policy).  One JSON line per (layer, splits): us, TFLOP/s.

    python tools/wgrad_sweep.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from singa_amd.ops import native as N

    L = N.lib()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    # (name, N, H, W, C, K, R, stride)
    shapes = [("s2_3x3", 1024, 28, 28, 128, 128, 3, 1), ("s3_3x3", 1024, 14, 14, 256, 256, 3, 1),
              ("s4_3x3", 1024, 7, 7, 512, 512, 3, 1), ("s3_conv1", 1024, 14, 14, 1024, 256, 1, 1),
              ("s2_conv1", 1024, 28, 28, 512, 128, 1, 1)]
    for name, Nn, H, W, C, K, R, st in shapes:
        p = R // 2
        Ho, Wo = (H + 2 * p - R) // st + 1, (W + 2 * p - R) // st + 1
        x = torch.randn(Nn, H, W, C, device="cuda").bfloat16()
        dy = torch.randn(Nn, Ho, Wo, K, device="cuda").bfloat16()
        dw = torch.zeros(K * R * R * C, device="cuda")
        flop = 2.0 * K * R * R * C * Nn * Ho * Wo
        for pol, sps in ((0, (0,)), (1, (0, 7, 8, 12, 14, 16, 21, 24, 28, 32, 48, 56, 64, 128))):
            L.set_tuning(13, pol)
            for sp in sps:
                L.set_tuning(12, sp)
                try:
                    f = lambda: L.conv_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), Nn, H, W, C, K, R, R, Ho,  # noqa
                                             Wo, st, st, p, p, 1, 1, 0, N.stream())
                    for _ in range(3):
                        f()
                    e0, e1 = ev(), ev()
                    torch.cuda.synchronize()
                    e0.record()
                    for _ in range(10):
                        f()
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) / 10 * 1e3
                finally:
                    L.set_tuning(12, 0)
                    L.set_tuning(13, 1)
                print(json.dumps({"layer": name, "policy": pol, "splits": sp, "us": round(us, 1),
                                  "TFs": round(flop / us * 1e-6, 1)}), flush=True)


if __name__ == "__main__":
    main()
