"""Per-shape convolution microbenchmark: singa_amd implicit-GEMM kernels vs
MIOpen (torch.nn.functional) for every distinct ResNet-50 conv at a given
batch.  Prints TFLOP/s for fwd / dgrad / wgrad."""
import argparse
import json
import sys
import os

import torch
import torch.nn.functional as TF

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from singa_amd.ops import functional as F  # noqa: E402
from singa_amd.ops import native as N  # noqa: E402

# (C, H, K, R, stride, count_in_resnet50)
SHAPES = [
    (8, 224, 64, 7, 2, 1),
    (64, 56, 64, 1, 1, 3), (64, 56, 64, 3, 1, 3), (64, 56, 256, 1, 1, 4), (256, 56, 64, 1, 1, 2),
    (256, 56, 128, 1, 1, 1), (128, 56, 128, 3, 2, 1), (128, 28, 512, 1, 1, 4), (256, 56, 512, 1, 2, 1),
    (512, 28, 128, 1, 1, 3), (128, 28, 128, 3, 1, 3),
    (512, 28, 256, 1, 1, 1), (256, 28, 256, 3, 2, 1), (256, 14, 1024, 1, 1, 6), (512, 28, 1024, 1, 2, 1),
    (1024, 14, 256, 1, 1, 5), (256, 14, 256, 3, 1, 5),
    (1024, 14, 512, 1, 1, 1), (512, 14, 512, 3, 2, 1), (512, 7, 2048, 1, 1, 3), (1024, 14, 2048, 1, 2, 1),
    (2048, 7, 512, 1, 1, 2), (512, 7, 512, 3, 1, 2),
]


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--no-miopen", action="store_true", help="skip the MIOpen (torch) yardstick")
    a = ap.parse_args()
    B = a.batch
    dev = torch.device("cuda")
    tot = {"ours": 0.0, "miopen": 0.0}
    for (C, H, K, R, st, cnt) in SHAPES:
        pad = R // 2
        x = torch.randn(B, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        Ho = (H + 2 * pad - R) // st + 1
        dy = torch.randn(B, K, Ho, Ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        flop = 2.0 * B * K * Ho * Ho * C * R * R
        dw = torch.zeros(K, C, R, R, device=dev).contiguous(memory_format=torch.channels_last)
        t_f = timeit(lambda: F.conv2d_fwd(x, w, None, (st, st), (pad, pad)))
        t_d = timeit(lambda: F.conv2d_bwd(x, w, dy, (st, st), (pad, pad), need_dx=True, dw_out=None)[0])
        t_w = timeit(lambda: F.conv2d_bwd(x, w, dy, (st, st), (pad, pad), need_dx=False, dw_out=dw))
        t_dw_only = t_w
        if a.no_miopen:
            m_f = m_d = m_w = float("nan")
        else:
            m_f = timeit(lambda: TF.conv2d(x, w, None, st, pad))
            m_d = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (st, st), (pad, pad), (1, 1),
                                                                     False, (0, 0), 1, (True, False, False)))
            m_w = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (st, st), (pad, pad), (1, 1),
                                                                     False, (0, 0), 1, (False, True, False)))
        ours = t_f + (t_d - t_dw_only if t_d > t_dw_only else t_d) + t_w
        # roofline: 2.5 PF dense bf16, 6.2 TB/s measured HBM copy ceiling (bw_probe_copy.jsonl)
        bx, by, bw_ = B * C * H * H * 2, B * K * Ho * Ho * 2, K * C * R * R * 2
        roof = lambda byts: max(flop / 2.5e12, byts / 6.2e9)  # noqa: E731  (ms)
        t_dg = max(t_d - t_w, 1e-6)
        rec = {"C": C, "H": H, "K": K, "R": R, "s": st, "n": cnt,
               "fwd_ms": round(t_f, 3), "dgrad+wgrad_ms": round(t_d, 3), "wgrad_ms": round(t_w, 3),
               "miopen_fwd_ms": round(m_f, 3), "miopen_dgrad_ms": round(m_d, 3), "miopen_wgrad_ms": round(m_w, 3),
               "fwd_TF": round(flop / t_f / 1e9, 1), "miopen_fwd_TF": round(flop / m_f / 1e9, 1),
               "dgrad_TF": round(flop / t_dg / 1e9, 1), "wgrad_TF": round(flop / t_w / 1e9, 1),
               "fwd_roof": round(roof(bx + by + bw_) / t_f, 2), "dgrad_roof": round(roof(bx + by + bw_) / t_dg, 2),
               "wgrad_roof": round(roof(bx + by + 2 * bw_) / t_w, 2),
               "step_ms": round(cnt * (t_f + t_d), 3)}
        tot["ours"] += cnt * (t_f + t_d)
        tot["miopen"] += cnt * (m_f + m_d + m_w)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_ms_per_step_convs": {k: round(v, 2) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
