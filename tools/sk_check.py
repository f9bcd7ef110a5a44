"""Correctness + timing of the persistent short-K GEMM (set_tuning(9, 1)) on
the 1x1-conv shapes, against igemm_k (knob off) and fp32 torch: plain bf16
output, beta accumulate, ragged M, and the conv-forward fused BN statistics."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from singa_amd.ops import functional as F  # noqa: E402
from singa_amd.ops import native as N  # noqa: E402


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
    return e0.elapsed_time(e1) / iters * 1e3


L = N.lib()
torch.manual_seed(0)
worst = 0.0
for (M, K, Nn) in ((262145, 64, 256), (200704, 128, 512), (300000, 72, 384), (3211264, 64, 256),
                   (802816, 128, 512), (200704, 64, 1024)):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(Nn, K, device="cuda").bfloat16()
    ref = (x[:8192].float() @ w.float().t())
    rec = {"M": M, "K": K, "N": Nn}
    outs = {}
    for knob in (0, 1):
        L.set_tuning(9, knob)
        o = F.gemm_nt(x, w, out_dtype=torch.bfloat16)
        outs[knob] = o
        rec[f"err{knob}"] = float((o[:8192].float() - ref).norm() / ref.norm())
        rec[f"us{knob}"] = round(timeit(lambda: F.gemm_nt(x, w, out_dtype=torch.bfloat16)), 1)
        # beta = 1 accumulate on top of a known C
        c0 = torch.randn(M, Nn, device="cuda").bfloat16()
        c = c0.clone()
        F.gemm(x, w, tb=True, out=c, beta=1.0)
        refb = ref + c0[:8192].float()
        rec[f"err_beta{knob}"] = float((c[:8192].float() - refb).norm() / refb.norm())
    rec["tail_rows_equal"] = bool(torch.equal(outs[0][-3:], outs[1][-3:]))
    worst = max(worst, rec["err1"], rec["err_beta1"])
    print(json.dumps(rec), flush=True)
    del x, w, c, c0, outs
    torch.cuda.empty_cache()
# conv forward with fused BN statistics (1x1, stride 1) -> batchnorm stats
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.randn(64, 64, 56, 56, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
w = (torch.randn(256, 64, 1, 1, device="cuda", generator=g) * 0.1).bfloat16().contiguous(
    memory_format=torch.channels_last)
res = []
for knob in (0, 1):
    L.set_tuning(9, knob)
    y = F.conv2d_fwd(x, w, None, (1, 1), (0, 0), out_dtype=torch.bfloat16, bn_stats=True)
    gam, bet = torch.ones(256, device="cuda"), torch.zeros(256, device="cuda")
    rm, rv = torch.zeros(256, device="cuda"), torch.ones(256, device="cuda")
    out, st = F.batchnorm_fwd(y, gam, bet, rm, rv, True, 0.1, 1e-5, relu=True)
    res.append((y.float(), st.mean.clone(), st.invstd.clone()))
L.set_tuning(9, 0)
e = [float((a - b).norm() / b.norm()) for a, b in zip(res[1], res[0])]
print(json.dumps({"conv_bn_stats_rel_err": e}))
worst = max([worst] + e)
print("worst", worst)
assert worst < 5e-3
