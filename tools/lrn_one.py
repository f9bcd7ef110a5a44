"""Time the LRN kernels on one activation shape against a same-size copy
(bandwidth yardstick); used for rocprofv3 --pmc passes too."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from singa_amd.ops import functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="512,96,55,55")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n, c, h, w = (int(v) for v in a.shape.split(","))
    dev = torch.device("cuda", 0)
    x = torch.randn(n, c, h, w, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn_like(x)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def t(fn):
        fn()
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(a.iters):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / a.iters * 1e3

    gb = x.numel() * 2 / 1e9
    rec = {"shape": a.shape, "GB": round(gb, 3),
           "copy_us": round(t(lambda: x.clone(memory_format=torch.channels_last)), 1),
           "fwd_us": round(t(lambda: F.lrn_fwd(x, 5, 1e-4, 0.75, 2.0)), 1),
           "bwd_us": round(t(lambda: F.lrn_bwd(x, dy, None, 5, 1e-4, 0.75, 2.0)), 1)}
    rec["fwd_TBps"] = round(2 * gb / rec["fwd_us"] * 1e3, 2)
    rec["bwd_TBps"] = round(3 * gb / rec["bwd_us"] * 1e3, 2)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
