"""Fused multi-head attention (csrc/kernels/fattn.hip) against an fp32
PyTorch reference of the same op: softmax(q k^T * scale + mask) v over the
in-place [B][S][3][H][D] projection, forward output and d(qkv), with and
without BERT's additive key mask; and the fused path inside a BERT encoder
layer against the unfused one (SINGA_AMD_FATTN=0)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(qkv, H, mask, scale, do):
    B, S, E = qkv.shape
    D = E // (3 * H)
    x = qkv.float().detach().requires_grad_(True)
    t = x.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
    s = torch.matmul(t[0], t[1].transpose(-1, -2)) * scale
    if mask is not None:
        s = s + mask.float()
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, t[2]).permute(0, 2, 1, 3).reshape(B, S, H * D)
    o.backward(do.float())
    return o.detach(), x.grad


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


@pytest.mark.parametrize("B,S,H", [(2, 128, 12), (3, 64, 4), (1, 32, 2), (4, 96, 3)])
@pytest.mark.parametrize("masked", [False, True])
def test_fused_attention_matches_fp32(gpu, B, S, H, masked):
    from singa_amd.ops import functional as F
    from singa_amd.ops import native as N

    D = 64
    assert N.lib().fattn_ok(S, D)
    g = torch.Generator(device=gpu).manual_seed(B * 1000 + S + H)
    qkv = (torch.randn(B, S, 3 * H * D, device=gpu, generator=g) * 0.8).bfloat16()
    do = torch.randn(B, S, H * D, device=gpu, generator=g).bfloat16()
    mask = None
    if masked:  # BERT's padding mask: the last keys of each sequence are padding
        keep = torch.ones(B, S, device=gpu)
        for b in range(B):
            keep[b, S - 1 - 7 * b:] = 0.0
        mask = ((1.0 - keep) * -10000.0).view(B, 1, 1, S)
    scale = 1.0 / math.sqrt(D)
    o, st = F.attention_qkv_fwd(qkv, H, mask, scale)
    assert isinstance(st, F.FAttnState)  # the fused path ran
    dq = F.attention_qkv_bwd(qkv, st, do, H, scale)
    o_ref, dq_ref = _ref(qkv, H, mask, scale, do)
    assert _rel(o, o_ref) < 1e-2, _rel(o, o_ref)
    HD = H * D
    for part, sl in (("dq", slice(0, HD)), ("dk", slice(HD, 2 * HD)), ("dv", slice(2 * HD, 3 * HD))):
        r = _rel(dq[..., sl], dq_ref[..., sl])
        assert r < 2e-2, (part, r)
    # the log-sum-exp the backward recomputes P from
    t = qkv.float().view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
    s = torch.matmul(t[0], t[1].transpose(-1, -2)) * scale
    if mask is not None:
        s = s + mask
    torch.testing.assert_close(st.lse.view(B, H, S), torch.logsumexp(s, -1), rtol=1e-3, atol=1e-3)
    # the projection's bias gradient summed on the way (accumulated into an
    # existing buffer); d(qkv) itself unchanged
    db0 = torch.randn(3 * HD, device=gpu, generator=g)
    db = db0.clone()
    dq2 = F.attention_qkv_bwd(qkv, st, do, H, scale, db_acc=db)
    assert torch.equal(dq2, dq)
    torch.testing.assert_close(db, db0 + dq.float().sum((0, 1)), rtol=1e-4, atol=1e-3)


def test_fused_attention_equals_unfused_path(gpu, monkeypatch):
    """The same op through the unfused path (two batched GEMMs + softmax
    kernels): both sit within bf16 rounding of each other."""
    from singa_amd.ops import functional as F

    B, S, H, D = 2, 128, 4, 64
    g = torch.Generator(device=gpu).manual_seed(7)
    qkv = torch.randn(B, S, 3 * H * D, device=gpu, generator=g).bfloat16()
    do = torch.randn(B, S, H * D, device=gpu, generator=g).bfloat16()
    o1, st = F.attention_qkv_fwd(qkv, H)
    d1 = F.attention_qkv_bwd(qkv, st, do, H)
    monkeypatch.setenv("SINGA_AMD_FATTN", "0")
    o2, p = F.attention_qkv_fwd(qkv, H)
    assert not isinstance(p, F.FAttnState)
    d2 = F.attention_qkv_bwd(qkv, p, do, H)
    assert _rel(o1, o2) < 1e-2 and _rel(d1, d2) < 3e-2, (_rel(o1, o2), _rel(d1, d2))


def test_bert_step_fused_vs_unfused(gpu, monkeypatch):
    """A small BERT trained 3 steps with and without the fused attention from
    the same init: the losses agree to bf16 accuracy."""
    import numpy as np

    from singa_amd import device, opt, tensor
    from singa_amd.models import bert

    def run(fused):
        monkeypatch.setenv("SINGA_AMD_FATTN", "1" if fused else "0")
        dev = device.create_rocm_gpu_on(0)
        dev.SetRandSeed(0)
        m = bert.Bert(vocab=500, hidden=128, layers=2, heads=2, ffn=256, max_pos=128, dropout=0.0,
                      compute_dtype=torch.bfloat16)
        rng = np.random.RandomState(0)
        ids = tensor.from_numpy(rng.randint(0, 500, (4, 64)).astype(np.int64), dev)
        y = tensor.from_numpy(rng.randint(0, 2, 4).astype(np.int32), dev)
        mk = np.ones((4, 64), np.float32)
        mk[1, 50:] = 0
        mask = tensor.from_numpy(mk, dev)
        m.set_optimizer(opt.Adam(1e-3))
        m.compile([ids], is_train=True)
        ls = []
        for _ in range(3):
            _, loss = m(ids, y, mask)
            ls.append(float(loss.data.float().cpu()))
        return ls

    a, b = run(True), run(False)
    np.testing.assert_allclose(a, b, rtol=2e-2, atol=2e-2)
