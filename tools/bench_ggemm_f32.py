"""fp32 generic-GEMM sweep (csrc/kernels/ggemm.hip) on the mlp.conf MLP shapes
(batch 1024, 784-2500-2000-1500-1000-500-10): forward (x @ W + b), data
gradient (dy @ W^T) and weight gradient (x^T @ dy, accumulate) under every
tile (``ggemm_tune(0, t)``: 1 64x64, 2 128x128 32x32x2, 3 128x64, 4 64x128,
5 128x128 16x16x4, 6 64x32, 7 32x64, 8 32x32) and split-K count (``ggemm_tune(1, s)``), plus a 4096^3
square.  Every configuration is checked against an fp64 reference before it
is timed.  One JSON line per (shape, kind, tile, splits); a summary of the
best configuration per shape at the end.

  python tools/bench_ggemm_f32.py [--tiles 1,2,3,4,5] [--splits -1,2,3,4,6,8]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from singa_amd.ops import functional as F  # noqa: E402
from singa_amd.ops import native as N  # noqa: E402

DIMS = (784, 2500, 2000, 1500, 1000, 500, 10)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--tiles", default="1,2,3,4,5,6,7,8")
    ap.add_argument("--splits", default="-1,2,3,4,6,8")
    ap.add_argument("--dma", default="0,-1", help="ggemm_tune(2, v): 0 the LDS-DMA kernel where it applies, -1 never")

    ap.add_argument("--square", type=int, default=4096)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    L = N.lib()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    B = a.batch
    tiles = [int(v) for v in a.tiles.split(",")]
    splits = [int(v) for v in a.splits.split(",")]
    dmas = [int(v) for v in a.dma.split(",")]
    shapes = []
    for i in range(len(DIMS) - 1):
        fin, fout = DIMS[i], DIMS[i + 1]
        x = torch.randn(B, fin, generator=g).to(dev)
        w = (torch.randn(fin, fout, generator=g) * 0.05).to(dev)
        b = torch.randn(fout, generator=g).to(dev)
        dy = torch.randn(B, fout, generator=g).to(dev)
        gw = torch.zeros(fin, fout, device=dev)
        shapes.append((f"fwd {B}x{fout}x{fin}", 2.0 * B * fin * fout,
                       lambda x=x, w=w, b=b: F.matmul(x, w, bias=b),
                       lambda x=x, w=w, b=b: x.double() @ w.double() + b.double()))
        if i > 0:
            shapes.append((f"dgrad {B}x{fin}x{fout}", 2.0 * B * fin * fout,
                           lambda dy=dy, w=w: F.gemm_nt(dy, w),
                           lambda dy=dy, w=w: dy.double() @ w.double().t()))
        # timed accumulating into gw; the check zeroes it first (``ref``)
        shapes.append((f"wgrad {fin}x{fout}x{B}", 2.0 * B * fin * fout,
                       lambda x=x, dy=dy, gw=gw: F.gemm_tn_acc(x, dy, gw),
                       lambda x=x, dy=dy, gw=gw: (gw.zero_(), x.double().t() @ dy.double())[1]))
    if a.square:
        S = a.square
        xa = torch.randn(S, S, generator=g).to(dev)
        xb = torch.randn(S, S, generator=g).to(dev)
        shapes.append((f"square {S}^3", 2.0 * S ** 3, lambda: F.matmul(xa, xb),
                       lambda: xa.double() @ xb.double()))
    out = open(a.out, "w") if a.out else None
    best = {}
    for name, flops, fn, ref in shapes:
        r = ref()
        scale = r.abs().max().item() + 1e-30
        for t, sp, dm in [(t, sp, dm) for t in tiles for sp in splits for dm in dmas]:
            if True:
                L.ggemm_tune(0, t)
                L.ggemm_tune(1, sp)
                L.ggemm_tune(2, dm)
                if name.startswith("square") and sp not in (-1, splits[0]):
                    continue
                if name.startswith("wgrad"):
                    ref()
                c = fn()
                torch.cuda.synchronize()
                err = (c.double() - r).abs().max().item() / scale
                us = timeit(fn)
                rec = {"shape": name, "tile": t, "splits": sp, "dma": L.ggemm_last_dma(), "us": round(us, 1),
                       "tflops": round(flops / us / 1e6, 1), "rel_err": float(f"{err:.2e}")}
                line = json.dumps(rec)
                print(line, flush=True)
                if out:
                    out.write(line + "\n")
                if err < 1e-5 and (name not in best or us < best[name]["us"]):
                    best[name] = rec
        L.ggemm_tune(0, 0)
        L.ggemm_tune(1, 0)
        L.ggemm_tune(2, 0)
        us = timeit(fn)
        rec = {"shape": name, "tile": "auto", "dma": L.ggemm_last_dma(), "us": round(us, 1),
               "tflops": round(flops / us / 1e6, 1)}
        print(json.dumps(rec), flush=True)
        best[name + " (auto)"] = rec
    print("# best per shape")
    tot_best = tot_auto = 0.0
    for k, v in best.items():
        print("#", k, json.dumps(v))
        if k.endswith("(auto)"):
            tot_auto += v["us"] if not k.startswith("square") else 0
        elif not k.startswith("square"):
            tot_best += v["us"]
    print(f"# MLP GEMM total: auto {tot_auto:.1f} us, best-per-shape {tot_best:.1f} us")


if __name__ == "__main__":
    main()
