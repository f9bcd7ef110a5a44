"""Fused transformer residual tail y = LayerNorm(x + dropout(a))
(autograd.DropAddLayerNorm, csrc/kernels/softmax.hip drop_add_ln_fwd_k /
layernorm_bwd2_k<DROP>) against a PyTorch fp32 reference of the same op (using
the kernel's own mask), and BERT with the fused op against the unfused
dropout -> add -> LayerNorm chain."""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("R,D", [(4096, 768), (37, 1024), (5, 40)])
def test_drop_add_ln_matches_fp32(gpu, dtype, R, D):
    from singa_amd.ops import functional as F

    g0 = torch.Generator(device=gpu).manual_seed(3)
    x = torch.randn(R, D, device=gpu, generator=g0).to(dtype)
    a = torch.randn(R, D, device=gpu, generator=g0).to(dtype)
    gam = torch.rand(D, device=gpu, generator=g0) + 0.5
    bet = torch.randn(D, device=gpu, generator=g0)
    ratio = 0.1
    y, s, mask, mu, rs = F.drop_add_layernorm_fwd(x, a, gam, bet, 1e-12, ratio, seed=11, offset=640)
    # the mask is the separate dropout kernel's stream for the same draw
    _, mask_ref = F.dropout_fwd(a, ratio, 11, 640)
    assert torch.equal(mask, mask_ref)
    keep = mask.float()
    xr = x.float().requires_grad_(True)
    ar = a.float().requires_grad_(True)
    gr, br = gam.clone().requires_grad_(True), bet.clone().requires_grad_(True)
    sr = xr + ar * keep / (1 - ratio)
    yr = TF.layer_norm(sr, (D,), gr, br, 1e-12)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel_err(y, yr.detach()) < tol and rel_err(s, sr.detach()) < tol
    dy = torch.randn(R, D, device=gpu, generator=g0).to(dtype)
    yr.backward(dy.float())
    dg, db = torch.zeros(D, device=gpu), torch.zeros(D, device=gpu)
    ds, da, dg, db, cs = F.drop_add_layernorm_bwd(s, dy, gam, mu, rs, mask, ratio, dg_acc=dg, db_acc=db)
    errs = {"dx": rel_err(ds, xr.grad), "da": rel_err(da, ar.grad), "dg": rel_err(dg, gr.grad),
            "db": rel_err(db, br.grad), "cs": rel_err(cs, da.float().sum(0))}
    print(errs)
    assert errs["dx"] < tol and errs["da"] < tol and errs["cs"] < 1e-5
    assert errs["dg"] < (1e-4 if dtype == torch.float32 else 2e-2) and errs["db"] < 1e-4


def test_bert_fused_tail_equals_unfused(gpu, monkeypatch):
    """BERT-tiny, same init and data: the fused residual tails reproduce the
    unfused chain's loss curve (same dropout masks) and really ran."""
    import numpy as np

    from singa_amd import autograd, device, opt, tensor
    from singa_amd.models import bert

    cfg = dict(vocab=1000, hidden=128, layers=2, heads=2, ffn=512, max_pos=128)
    rng = np.random.RandomState(0)
    ids_np = rng.randint(0, cfg["vocab"], (8, 64)).astype(np.int64)
    y_np = rng.randint(0, 2, 8).astype(np.int32)
    calls = [0]
    orig = autograd.DropAddLayerNorm.forward

    def spy(self, *a):
        calls[0] += 1
        return orig(self, *a)

    monkeypatch.setattr(autograd.DropAddLayerNorm, "forward", spy)
    # the unfused attention in both arms: this compares the residual tails
    # alone (the fused attention is checked in test_fattn_gpu.py)
    monkeypatch.setenv("SINGA_AMD_FATTN", "0")
    # and the separate gradient adds in both (the in-place accumulation into
    # the tail's ds rounds once instead of twice: test_linear_dgrad_accumulates_...)
    monkeypatch.setattr(autograd, "INPLACE_ACC", False)
    curves, init = {}, None
    for fused in ("1", "0"):
        monkeypatch.setenv("SINGA_AMD_FUSED_DAL", fused)
        dev = device.create_rocm_gpu()
        dev.SetRandSeed(0)
        m = bert.Bert(dropout=0.1, compute_dtype=torch.bfloat16, **cfg)
        ids = tensor.from_numpy(ids_np, dev)
        y = tensor.from_numpy(y_np, dev)
        m.set_optimizer(opt.Adam(1e-4))
        m.compile([ids], is_train=True, use_graph=False)
        if init is None:
            init = {k: v.data.float().clone() for k, v in m.get_states().items()}
        else:
            m.set_states({k: v.to(m.get_states()[k].data.dtype) for k, v in init.items()})
        dev.SetRandSeed(5)
        m.train()
        ls = []
        for _ in range(4):
            _, loss = m(ids, y)
            ls.append(float(loss.data.float().cpu()))
        curves[fused] = ls
        if fused == "1":
            assert calls[0] >= 4 * 2 * cfg["layers"]
            n_fused = calls[0]
    assert calls[0] == n_fused  # the unfused run did not take it
    print(curves)
    np.testing.assert_allclose(curves["1"], curves["0"], rtol=2e-3)


def test_producer_bias_gradient_summed_in_place(gpu, monkeypatch):
    """The residual tail's backward sums da's columns straight into the
    producing Linear's bias gradient (no temporary + add): one SGD step
    (lr 1, so w0 - w1 is the gradient) equals the path that hands the sums
    to the Linear, and the in-place route really ran."""
    import numpy as np

    from singa_amd import autograd, device, opt, tensor
    from singa_amd.models import bert

    cfg = dict(vocab=1000, hidden=128, layers=2, heads=2, ffn=512, max_pos=128)
    rng = np.random.RandomState(1)
    ids_np = rng.randint(0, cfg["vocab"], (8, 64)).astype(np.int64)
    y_np = rng.randint(0, 2, 8).astype(np.int32)
    orig = autograd.DropAddLayerNorm._producer_bias
    taken = [0]

    def spy(self):
        r = orig(self)
        taken[0] += r[1] is not None
        return r

    res, init = {}, None
    for arm in ("inplace", "handoff"):
        monkeypatch.setattr(autograd.DropAddLayerNorm, "_producer_bias",
                            spy if arm == "inplace" else (lambda self: (None, None)))
        dev = device.create_rocm_gpu()
        dev.SetRandSeed(0)
        m = bert.Bert(dropout=0.1, compute_dtype=torch.bfloat16, **cfg)
        ids = tensor.from_numpy(ids_np, dev)
        y = tensor.from_numpy(y_np, dev)
        m.set_optimizer(opt.SGD(lr=1.0))
        m.compile([ids], is_train=True, use_graph=False)
        if init is None:
            init = {k: v.data.float().clone() for k, v in m.get_states().items()}
        else:
            m.set_states({k: v.to(m.get_states()[k].data.dtype) for k, v in init.items()})
        dev.SetRandSeed(5)
        m.train()
        m(ids, y)
        res[arm] = {k: init[k] - v.data.float() for k, v in m.get_params().items()}
    assert taken[0] == 2 * cfg["layers"]  # proj and fc2 of every layer
    worst = max(rel_err(res["inplace"][k], res["handoff"][k]) for k in res["handoff"]
                if float(res["handoff"][k].norm()) > 0)
    assert worst < 1e-4, worst


def test_fc1_bias_gradient_from_fc2_dgrad_epilogue(gpu, monkeypatch):
    """fc1's bias gradient summed in fc2's data-gradient epilogue (the GEMM
    that applies fc1's GELU backward): one SGD step equals the path with the
    separate column-sum pass (SINGA_AMD_BIAS_INPLACE=0 equivalent)."""
    import numpy as np

    from singa_amd import autograd, device, opt, tensor
    from singa_amd.models import bert

    cfg = dict(vocab=1000, hidden=128, layers=2, heads=2, ffn=512, max_pos=128)
    rng = np.random.RandomState(2)
    ids_np = rng.randint(0, cfg["vocab"], (8, 64)).astype(np.int64)
    y_np = rng.randint(0, 2, 8).astype(np.int32)
    res, init = {}, None
    for on in (True, False):
        monkeypatch.setattr(autograd, "BIAS_INPLACE", on)
        dev = device.create_rocm_gpu()
        dev.SetRandSeed(0)
        m = bert.Bert(dropout=0.0, compute_dtype=torch.bfloat16, **cfg)
        ids = tensor.from_numpy(ids_np, dev)
        y = tensor.from_numpy(y_np, dev)
        m.set_optimizer(opt.SGD(lr=1.0))
        m.compile([ids], is_train=True, use_graph=False)
        if init is None:
            init = {k: v.data.float().clone() for k, v in m.get_states().items()}
        else:
            m.set_states({k: v.to(m.get_states()[k].data.dtype) for k, v in init.items()})
        m.train()
        m(ids, y)
        res[on] = {k: init[k] - v.data.float() for k, v in m.get_params().items()}
    worst = max(rel_err(res[True][k], res[False][k]) for k in res[False] if float(res[False][k].norm()) > 0)
    assert worst < 1e-4, worst


def test_linear_dgrad_accumulates_into_residual_gradient(gpu, monkeypatch):
    """The q/k/v and fc1 projections' data gradients add into the residual
    tail's pending gradient of their shared input in the GEMM epilogue (beta
    1, one bf16 rounding instead of two): one SGD step matches the separate
    add pass (autograd.INPLACE_ACC off) to bf16 accuracy, and the in-place
    route really ran."""
    import numpy as np

    from singa_amd import autograd, device, opt, tensor
    from singa_amd.models import bert
    from singa_amd.ops import functional as F

    cfg = dict(vocab=1000, hidden=128, layers=2, heads=2, ffn=512, max_pos=128)
    rng = np.random.RandomState(4)
    ids_np = rng.randint(0, cfg["vocab"], (8, 64)).astype(np.int64)
    y_np = rng.randint(0, 2, 8).astype(np.int32)
    orig = F.gemm
    n_beta1 = [0]

    def spy(*a, **kw):
        n_beta1[0] += kw.get("beta", 0.0) == 1.0 and kw.get("out") is not None and kw.get("out").dtype == torch.bfloat16
        return orig(*a, **kw)

    monkeypatch.setattr(F, "gemm", spy)
    res, init = {}, None
    for on in (True, False):
        monkeypatch.setattr(autograd, "INPLACE_ACC", on)
        dev = device.create_rocm_gpu()
        dev.SetRandSeed(0)
        m = bert.Bert(dropout=0.0, compute_dtype=torch.bfloat16, **cfg)
        ids = tensor.from_numpy(ids_np, dev)
        y = tensor.from_numpy(y_np, dev)
        m.set_optimizer(opt.SGD(lr=1.0))
        m.compile([ids], is_train=True, use_graph=False)
        if init is None:
            init = {k: v.data.float().clone() for k, v in m.get_states().items()}
        else:
            m.set_states({k: v.to(m.get_states()[k].data.dtype) for k, v in init.items()})
        m.train()
        n0 = n_beta1[0]
        m(ids, y)
        if on:
            assert n_beta1[0] - n0 >= 2 * cfg["layers"]  # q/k/v and fc1 of every layer
        res[on] = {k: init[k] - v.data.float() for k, v in m.get_params().items()}
    worst = max(rel_err(res[True][k], res[False][k]) for k in res[False] if float(res[False][k].norm()) > 0)
    assert worst < 2e-2, worst


def test_gelu_backward_in_fc2_dgrad_epilogue(gpu, monkeypatch):
    """fc2's data-gradient GEMM applies the standalone GELU's derivative in its
    epilogue (and sums fc1's bias gradient there): one SGD step equals the
    separate GELU-backward / column-sum passes, and the fused route ran."""
    import numpy as np

    from singa_amd import autograd, device, opt, tensor
    from singa_amd.models import bert
    from singa_amd.ops import functional as F

    cfg = dict(vocab=1000, hidden=128, layers=2, heads=2, ffn=512, max_pos=128)
    rng = np.random.RandomState(6)
    ids_np = rng.randint(0, cfg["vocab"], (8, 64)).astype(np.int64)
    y_np = rng.randint(0, 2, 8).astype(np.int32)
    orig = F.unary_bwd
    n_gelu_bwd = [0]

    def spy(kind, *a, **kw):
        n_gelu_bwd[0] += kind == "gelu"
        return orig(kind, *a, **kw)

    monkeypatch.setattr(F, "unary_bwd", spy)
    monkeypatch.setenv("SINGA_AMD_FUSE_GELU", "0")
    res, init, counts = {}, None, {}
    for on in (True, False):
        monkeypatch.setattr(autograd, "ACT_GRAD_FUSE", on)
        dev = device.create_rocm_gpu()
        dev.SetRandSeed(0)
        m = bert.Bert(dropout=0.0, compute_dtype=torch.bfloat16, **cfg)
        ids = tensor.from_numpy(ids_np, dev)
        y = tensor.from_numpy(y_np, dev)
        m.set_optimizer(opt.SGD(lr=1.0))
        m.compile([ids], is_train=True, use_graph=False)
        if init is None:
            init = {k: v.data.float().clone() for k, v in m.get_states().items()}
        else:
            m.set_states({k: v.to(m.get_states()[k].data.dtype) for k, v in init.items()})
        m.train()
        n0 = n_gelu_bwd[0]
        m(ids, y)
        counts[on] = n_gelu_bwd[0] - n0
        res[on] = {k: init[k] - v.data.float() for k, v in m.get_params().items()}
    assert counts[True] == 0 and counts[False] >= cfg["layers"], counts
    worst = max(rel_err(res[True][k], res[False][k]) for k in res[False] if float(res[False][k].norm()) > 0)
    assert worst < 2e-2, worst
