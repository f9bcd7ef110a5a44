"""Per-call time of BERT-base's elementwise / normalisation kernels at the
bench shape (32 x 128 tokens: [4096, 768] and [4096, 3072] bf16), against a
device copy of the same bytes and PyTorch's own HIP kernels as yardsticks.
One JSON line per op: {"op", "us", "GBps"}.

    python tools/bert_elem_bench.py [--iters 200]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as TF

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    from singa_amd.ops import functional as F
    from singa_amd.ops import glue as G
    from singa_amd.ops import native as N

    torch.cuda.set_stream(torch.cuda.ExternalStream(N.stream()) if isinstance(N.stream(), int) else
                          torch.cuda.current_stream())
    g0 = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(4096, 768, device="cuda", generator=g0).bfloat16()
    r = torch.randn(4096, 768, device="cuda", generator=g0).bfloat16()
    dy = torch.randn(4096, 768, device="cuda", generator=g0).bfloat16()
    h = torch.randn(4096, 3072, device="cuda", generator=g0).bfloat16()
    dh = torch.randn(4096, 3072, device="cuda", generator=g0).bfloat16()
    gam = torch.rand(768, device="cuda", generator=g0) + 0.5
    bet = torch.randn(768, device="cuda", generator=g0)
    _, mu, rs = F.layernorm_fwd(x, gam, bet)
    dg, db = torch.zeros(768, device="cuda"), torch.zeros(768, device="cuda")
    out_s, out_l = torch.empty_like(x), torch.empty_like(h)
    def _v1(fn):
        F.LNB_V2 = False
        try:
            return fn()
        finally:
            F.LNB_V2 = True

    mb = lambda *ts: sum(t.numel() * t.element_size() for t in ts) / 1e6  # noqa: E731
    cases = [
        ("copy_4096x768", lambda: G.copy_(out_s, x), mb(x, out_s)),
        ("copy_4096x3072", lambda: G.copy_(out_l, h), mb(h, out_l)),
        ("ln_fwd", lambda: F.layernorm_fwd(x, gam, bet), mb(x, x)),
        ("ln_bwd", lambda: F.layernorm_bwd(x, dy, gam, mu, rs, dg_acc=dg, db_acc=db), mb(x, dy, x)),
        ("ln_bwd_v1", lambda: _v1(lambda: F.layernorm_bwd(x, dy, gam, mu, rs, dg_acc=dg, db_acc=db)), mb(x, dy, x)),
        ("gelu_fwd", lambda: F.unary("gelu", h), mb(h, h)),
        ("gelu_bwd", lambda: F.unary_bwd("gelu", h, None, dh), mb(h, dh, h)),
        ("add_act", lambda: F.add_act(x, r), mb(x, r, x)),
        ("torch_layer_norm", lambda: TF.layer_norm(x, (768,), gam.bfloat16(), bet.bfloat16()), mb(x, x)),
        ("torch_gelu", lambda: TF.gelu(h), mb(h, h)),
    ]
    for name, fn, m in cases:
        us = timeit(fn, a.iters)
        print(json.dumps({"op": name, "us": round(us, 2), "GBps": round(m / us * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
