"""Time the ResNet-50 stride-2 3x3 data gradients (stage transitions, b1024:
C = K = 128 / 256 / 512 from 56 / 28 / 14 to 28 / 14 / 7) with the identity-sum
masked-sum epilogue, under the tuning knobs in SG_TUNE (A/B of tile choices
for the four stride phases).  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from singa_amd.ops import native as N  # noqa: E402


def main():
    L = N.lib()
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("BATCH", "1024"))
    for c, h in ((128, 56), (256, 28), (512, 14)):
        ho = h // 2
        dy = torch.randn(n, ho, ho, c, device=dev).bfloat16()
        w = (torch.randn(c, 3, 3, c, device=dev) * 0.02).bfloat16()
        dx = torch.empty(n, h, h, c, device=dev, dtype=torch.bfloat16)
        wt = torch.empty(c * c * 9, device=dev, dtype=torch.bfloat16)
        ws = torch.zeros(32 * 2 * c, device=dev)
        mask = torch.randint(0, 256, (n * h * h * c // 8,), device=dev, dtype=torch.uint8)

        def f():
            L.conv_dgrad_bn(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), n, h, h, c, c, 3, 3, ho, ho, 2, 2, 1, 1, 1, 1,
                            wt.data_ptr(), ws.data_ptr(), 0, 0, 0, 0, 0, N.stream(), 0.0, mask.data_ptr())
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        fl = 2.0 * n * ho * ho * c * c * 9
        print(json.dumps({"shape": f"dgrad 3x3/s2 C{c} {h}->{ho}", "tune": os.environ.get("SG_TUNE", ""),
                          "ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
