"""Run one conv pass repeatedly (for rocprofv3 counter collection).
    python tools/conv_one.py --C 256 --H 14 --K 256 --R 3 --s 1 --batch 256 --pass fwd --iters 20"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from singa_amd.ops import functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    for k, d in (("C", 256), ("H", 14), ("K", 256), ("R", 3), ("s", 1), ("batch", 256), ("iters", 20)):
        ap.add_argument(f"--{k}", type=int, default=d)
    ap.add_argument("--pass", dest="which", default="fwd")
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, C, H, K, R, st = a.batch, a.C, a.H, a.K, a.R, a.s
    pad = R // 2
    x = torch.randn(B, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 * pad - R) // st + 1
    dy = torch.randn(B, K, Ho, Ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dw = torch.zeros(K, C, R, R, device=dev).contiguous(memory_format=torch.channels_last)
    for _ in range(a.iters):
        if a.which == "fwd":
            F.conv2d_fwd(x, w, None, (st, st), (pad, pad))
        elif a.which == "dgrad":
            F.conv2d_bwd(x, w, dy, (st, st), (pad, pad), need_dx=True, dw_out=None)
        else:
            F.conv2d_bwd(x, w, dy, (st, st), (pad, pad), need_dx=False, dw_out=dw)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
