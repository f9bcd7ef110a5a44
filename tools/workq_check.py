"""Exactness check of the persistent kernels' dynamic work queues at the
ResNet-50 b1024 shapes: static partition vs queue vs a PyTorch fp32
reference of the same 1x1 convolution, output NaN-filled before each launch
(a skipped tile stays NaN).  One JSON line per (shape, stats, path)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from singa_amd.ops import native as N  # noqa: E402


def main():
    L = N.lib()
    dev = torch.device("cuda", 0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    for (h, c, k) in ((56, 64, 256), (28, 128, 512), (14, 128, 512)):
        x = torch.randn(n, h, h, c, device=dev).bfloat16()
        w = (torch.randn(k, 1, 1, c, device=dev) * 0.1).bfloat16()
        ref = (x.float().reshape(-1, c) @ w.float().reshape(k, c).t()).reshape(n, h, h, k)
        y = torch.empty(n, h, h, k, device=dev, dtype=torch.bfloat16)
        ws = torch.zeros(32 * 2 * k, dtype=torch.float32, device=dev)
        for stats in (0, 1):
            for q in (0, 1, 1):
                L.workq_set(q)
                y.fill_(float("nan"))
                ws.zero_()
                L.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, n, h, h, c, k, 1, 1, h, h, 1, 1, 0, 0, 1, 1,
                           0, 0, N.stream(), ws.data_ptr() if stats else 0)
                torch.cuda.synchronize()
                yf = y.float()
                nan_rows = int(torch.isnan(yf).reshape(-1, k).any(1).sum())
                err = float(((yf - ref).abs().nan_to_num(1e9).max()))
                print(json.dumps({"shape": [n, h, h, c, k], "stats": stats, "queue": q, "nan_rows": nan_rows,
                                  "max_abs_err": err, "ref_max": float(ref.abs().max())}), flush=True)
    L.workq_set(1)


if __name__ == "__main__":
    main()
