"""Would running a conv's weight gradient concurrently with its data gradient
(two HIP streams) beat running them back to back?  Per ResNet-50 b1024 conv
shape: mean time of dgrad + wgrad serial on one stream vs the two forked onto
two streams (independent outputs), plus each alone.

    python tools/probe_overlap.py [--iters 10] [--out profiles/r6/probe_overlap.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from singa_amd.ops import native as N  # noqa: E402

# (name, N, C, H, K, R, stride)
SHAPES = [("s1_1x1_64_256", 1024, 64, 56, 256, 1, 1), ("s1_1x1_256_64", 1024, 256, 56, 64, 1, 1),
          ("s2_3x3_128", 1024, 128, 28, 128, 3, 1), ("s3_3x3_256", 1024, 256, 14, 256, 3, 1),
          ("s4_3x3_512", 1024, 512, 7, 512, 3, 1), ("s3_1x1_256_1024", 1024, 256, 14, 1024, 1, 1),
          ("s3_1x1_1024_256", 1024, 1024, 14, 256, 1, 1), ("s4_1x1_2048_512", 1024, 2048, 7, 512, 1, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    L = N.lib()
    dev = torch.device("cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    recs = []
    for name, n, c, h, k, r, st in SHAPES:
        p = r // 2
        ho = (h + 2 * p - r) // st + 1
        x = torch.randn(n, c, h, h, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(k, c, r, r, device=dev) * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, k, ho, ho, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        wt = torch.empty(k * c * r * r, device=dev, dtype=torch.bfloat16)  # K-major weights (transposed per call)
        dw = torch.zeros(k, c, r, r, device=dev).contiguous(memory_format=torch.channels_last)
        args = (n, h, h, c, k, r, r, ho, ho, st, st, p, p, 1, 1)

        def dgrad(s):
            L.conv_dgrad_acc(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), *args, 0, 0.0, s.cuda_stream, wt.data_ptr())

        def wgrad(s):
            L.conv_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *args, 0, s.cuda_stream)

        def timed(fn):
            torch.cuda.synchronize()
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            cur = torch.cuda.current_stream()
            e0.record(cur)
            for _ in range(a.iters):
                fn()
            e1.record(cur)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / a.iters

        def serial():
            cur = torch.cuda.current_stream()
            dgrad(cur)
            wgrad(cur)

        def forked():
            cur = torch.cuda.current_stream()
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            dgrad(s1)
            wgrad(s2)
            cur.wait_stream(s1)
            cur.wait_stream(s2)

        rec = {"shape": name, "dgrad_us": round(timed(lambda: dgrad(torch.cuda.current_stream())), 1),
               "wgrad_us": round(timed(lambda: wgrad(torch.cuda.current_stream())), 1),
               "serial_us": round(timed(serial), 1), "forked_us": round(timed(forked), 1)}
        rec["gain"] = round(1.0 - rec["forked_us"] / rec["serial_us"], 4)
        recs.append(rec)
        print(json.dumps(rec), flush=True)
        del x, w, dy, dx, dw, wt
    if a.out:
        with open(a.out, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
