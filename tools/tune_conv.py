"""Sweep the conv tuning knobs (native ``set_tuning``) per ResNet-50 shape;
prints ms per pass and the step-weighted totals for each policy.

    python tools/tune_conv.py --batch 256 --knob 0 --values 0,1,2,3 --pass wgrad
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from singa_amd.ops import functional as F  # noqa: E402
from singa_amd.ops import native as N  # noqa: E402
from tools.bench_conv import SHAPES, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--knob", type=int, default=0)
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--pass", dest="which", default="wgrad", choices=["fwd", "dgrad", "wgrad", "dx"])
    ap.add_argument("--set", default="", help="fixed knobs for the whole sweep, e.g. 2=1,3=0")
    a = ap.parse_args()
    for kv in filter(None, a.set.split(",")):
        k, v = kv.split("=")
        N.lib().set_tuning(int(k), int(v))
    vals = [int(v) for v in a.values.split(",")]
    B = a.batch
    dev = torch.device("cuda")
    tot = {v: 0.0 for v in vals}
    for (C, H, K, R, st, cnt) in SHAPES:
        pad = R // 2
        x = torch.randn(B, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        Ho = (H + 2 * pad - R) // st + 1
        dy = torch.randn(B, K, Ho, Ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dw = torch.zeros(K, C, R, R, device=dev).contiguous(memory_format=torch.channels_last)
        flop = 2.0 * B * K * Ho * Ho * C * R * R
        row = {"C": C, "H": H, "K": K, "R": R, "s": st, "n": cnt}
        ref = None
        for v in vals:
            N.lib().set_tuning(a.knob, v)
            if a.which == "wgrad":
                dw.zero_()
                F.conv2d_bwd(x, w, dy, (st, st), (pad, pad), need_dx=False, dw_out=dw)
                out = dw.clone()
                t = timeit(lambda: F.conv2d_bwd(x, w, dy, (st, st), (pad, pad), need_dx=False, dw_out=dw))
            elif a.which == "dx":  # data gradient only (the native kernel, no weight gradient)
                dx = torch.empty_like(x)

                wt = torch.empty(K * C * R * R, dtype=torch.bfloat16, device=dev)

                def run():  # knob 5 (tools-only): 1 = K-major transposed-weight path
                    N.lib().conv_dgrad_acc(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), B, H, H, C, K, R, R, Ho, Ho,
                                           st, st, pad, pad, 1, 1, 0, 0.0, N.stream(),
                                           wt.data_ptr() if (a.knob == 5 and v == 1) else 0)
                    return dx
                out = run().float().clone()
                t = timeit(run)
            elif a.which == "dgrad":
                out = F.conv2d_bwd(x, w, dy, (st, st), (pad, pad), need_dx=True, dw_out=None)[0].float()
                t = timeit(lambda: F.conv2d_bwd(x, w, dy, (st, st), (pad, pad), need_dx=True, dw_out=None)[0])
            else:
                out = F.conv2d_fwd(x, w, None, (st, st), (pad, pad)).float()
                t = timeit(lambda: F.conv2d_fwd(x, w, None, (st, st), (pad, pad)))
            if ref is None:
                ref = out
            err = float((out - ref).abs().max() / (ref.abs().max() + 1e-6))
            row[f"ms_{v}"] = round(t, 4)
            row[f"TF_{v}"] = round(flop / t / 1e9, 1)
            row[f"err_{v}"] = round(err, 5)
            tot[v] += t * cnt
        print(json.dumps(row), flush=True)
    print(json.dumps({"total_ms_weighted": {str(k): round(v, 3) for k, v in tot.items()}}))
    N.lib().set_tuning(a.knob, {0: 5, 1: 1, 2: 1}.get(a.knob, 0))  # restore the default


if __name__ == "__main__":
    main()
