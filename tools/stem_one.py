"""Run the paired-tap ResNet stem conv (forward or weight gradient) repeatedly
(for rocprofv3 counter collection): python tools/stem_one.py --pass fwd --batch 1024"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from singa_amd.ops import native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pass", dest="which", default="fwd")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    L = N.lib()
    dev = torch.device("cuda")
    B, H, W, K = a.batch, 224, 224, 64
    xp = torch.randn(B, H, W + 1, 8, device=dev).to(torch.bfloat16)
    wp = (torch.randn(K * 7 * 4 * 8, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty(B, 112, 112, K, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(K * 7 * 4 * 8, device=dev)
    for _ in range(a.iters):
        if a.which == "fwd":
            L.conv_fwd(xp.data_ptr(), wp.data_ptr(), y.data_ptr(), 0, B, H, W + 1, 8, K, 7, 4, 112, 112, 2, 2, 3, 2, 1,
                       2, 0, 0, N.stream(), 0)
        else:
            L.conv_wgrad(xp.data_ptr(), y.data_ptr(), dw.data_ptr(), B, H, W + 1, 8, K, 7, 4, 112, 112, 2, 2, 3, 2, 1,
                         2, 0, N.stream())
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
