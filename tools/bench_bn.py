"""HBM-bandwidth microbenchmark of the BatchNorm apply kernels (forward
bn_apply with ReLU + 1-bit mask, with/without residual; backward apply with
mask bits + residual gradient) on ResNet-50 activation shapes, for each
(rows per thread of a workgroup's contiguous row span, rows-per-iteration
unroll) pair: rpt 0 = the legacy grid-stride walk over <= 2048 workgroups
(bn_set_rows_per_thread, bn_set_unroll).  Prints achieved GB/s next to a
torch copy of the same tensor as the yardstick."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from singa_amd.ops import native as N  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default="")
    ap.add_argument("--configs", default="0:1,0:2,2:1,4:1,4:2,8:2,16:2", help="rpt:ur pairs")
    a = ap.parse_args()
    L = N.lib()
    dev = torch.device("cuda:0")
    rows = []
    for (H, C) in [(112, 64), (56, 64), (56, 256), (28, 128), (28, 512), (14, 256), (14, 1024), (7, 512), (7, 2048)]:
        R = a.batch * H * H
        x = torch.randn(R, C, device=dev).to(torch.bfloat16)
        res = torch.randn(R, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(R, C, device=dev).to(torch.bfloat16)
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x)
        mask = torch.empty(R * C // 8, dtype=torch.uint8, device=dev)
        f = lambda n: torch.rand(n, device=dev)  # noqa: E731
        scale, shift, mean, invstd, gamma = f(C), f(C), f(C), f(C), f(C)
        ws = torch.zeros(2 * C, device=dev)
        coef, dg, db = f(3 * C), torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        eb = R * C * 2
        t_copy = timeit(lambda: y.copy_(x))
        rec = {"H": H, "C": C, "R": R, "copy_GBs": round(2 * eb / t_copy / 1e9)}
        for cfg in a.configs.split(","):
            rpt, ur = map(int, cfg.split(":"))
            L.bn_set_rows_per_thread(rpt)
            L.bn_set_unroll(ur)
            t1 = timeit(lambda: L.bn_apply(x.data_ptr(), scale.data_ptr(), shift.data_ptr(), 0, y.data_ptr(), R, C, 1,
                                           N.dt(x), N.stream(), mask.data_ptr()))
            t2 = timeit(lambda: L.bn_apply(x.data_ptr(), scale.data_ptr(), shift.data_ptr(), res.data_ptr(),
                                           y.data_ptr(), R, C, 1, N.dt(x), N.stream(), mask.data_ptr()))
            t3 = timeit(lambda: L.bn_bwd_from_ws(x.data_ptr(), dy.data_ptr(), mask.data_ptr(), scale.data_ptr(),
                                                 shift.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                                 gamma.data_ptr(), ws.data_ptr(), 1, coef.data_ptr(), dg.data_ptr(),
                                                 db.data_ptr(), dx.data_ptr(), dres.data_ptr(), R, C, 3, N.dt(x),
                                                 N.stream()))
            rec[f"rpt{rpt}_ur{ur}"] = {"fwd_GBs": round((2 * eb + eb / 16) / t1 / 1e9),
                              "fwd_res_GBs": round((3 * eb + eb / 16) / t2 / 1e9),
                              "bwd_GBs": round((4 * eb + eb / 16) / t3 / 1e9),
                              "us": [round(t * 1e6, 1) for t in (t1, t2, t3)]}
        L.bn_set_unroll(0)
        L.bn_set_rows_per_thread(4)
        print(json.dumps(rec), flush=True)
        rows.append(rec)
        del x, res, dy, y, dx, dres, mask
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
