"""Cost of the masked-gradient sum (stats_mode 3) in the conv dgrad epilogue:
plain dgrad vs dgrad + sum(g~) from mask bits, per ResNet-50 consumer shape
(3x3 conv2 and 1x1 conv3 of a bottleneck) at batch 1024."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from singa_amd.ops import native as N  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


L = N.lib()
B = 1024
for (C, H, K, R, st) in ((64, 56, 64, 3, 1), (64, 56, 256, 1, 1), (128, 28, 128, 3, 1), (128, 28, 512, 1, 1),
                         (128, 56, 128, 3, 2), (256, 14, 256, 3, 1), (256, 14, 1024, 1, 1)):
    pad = R // 2
    Ho = (H + 2 * pad - R) // st + 1
    dy = torch.randn(B * Ho * Ho * K, device="cuda").bfloat16()
    w = (torch.randn(K * R * R * C, device="cuda") * 0.05).bfloat16()
    dx = torch.empty(B * H * H * C, device="cuda").bfloat16()
    wt = torch.empty(K * R * R * C, device="cuda").bfloat16()
    mask = torch.randint(0, 255, (B * H * H * C // 8,), device="cuda", dtype=torch.uint8)
    ws = torch.zeros(32 * 2 * C, device="cuda")
    s = N.stream()

    def plain():
        L.conv_dgrad_acc(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), B, H, H, C, K, R, R, Ho, Ho, st, st, pad, pad, 1, 1,
                         0, 0.0, s, wt.data_ptr())

    def gsum():
        L.conv_dgrad_bn(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), B, H, H, C, K, R, R, Ho, Ho, st, st, pad, pad, 1, 1,
                        wt.data_ptr(), ws.data_ptr(), 0, 0, 0, 0, 0, s, 0.0, mask.data_ptr())
    rec = {"C": C, "H": H, "K": K, "R": R, "s": st, "us_plain": round(timeit(plain), 1),
           "us_gsum": round(timeit(gsum), 1)}
    print(json.dumps(rec), flush=True)
    del dy, w, dx, wt, mask
    torch.cuda.empty_cache()
