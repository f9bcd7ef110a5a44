"""The CppCPU device's native C++ compute backend (csrc/runtime/cpu_ops.cc via
singa_amd/ops/cpu.py) against the PyTorch-CPU oracle (``cpu.torch_oracle()``).

* BASELINE config #1 (MLP 784-512-10) and the reference's LeNet conf
  (examples/mnist/conv.conf, reference examples/mnist/conv.conf) train with a
  guard that FAILS on any torch compute call -- only allocation, metadata and
  free views may reach PyTorch -- and match the oracle run to 1e-5;
* per-op parity of every native kernel (GEMM orientations / batches /
  epilogues, grouped / dilated / strided convolution, pooling, LRN, softmax
  cross-entropy, batch / layer norm, the unary table, broadcast binary,
  where, reductions, casts, gathers, padding, dropout).
Reference semantics: include/mshadow/tensor_cpu-inl.hpp:52-165,
src/worker/layer.cc:18-764."""
import collections
import os
import traceback

import numpy as np
import pytest
import torch
import torch.nn.functional as TF
from torch.overrides import TorchFunctionMode

from singa_amd.ops import cpu as CP
from singa_amd.ops import functional as F
from singa_amd.ops import glue as G

pytestmark = pytest.mark.skipif(CP.lib() is None, reason="_core runtime not built")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# PyTorch calls that move no data through a PyTorch kernel
_ALLOW = {"__get__", "dim", "size", "stride", "numel", "data_ptr", "element_size", "is_contiguous", "view",
          "as_strided", "permute", "transpose", "t", "unsqueeze", "squeeze", "expand", "movedim", "narrow",
          "__getitem__", "numpy", "detach", "requires_grad_", "_set_grad_enabled", "empty", "empty_like",
          "empty_strided", "storage_offset", "untyped_storage", "__len__", "__hash__", "__eq__", "is_floating_point",
          "unbind", "split", "chunk", "from_numpy", "__format__", "__repr__", "tolist", "item", "__float__",
          "__int__", "__bool__", "__index__", "view_as", "get_device", "is_complex", "has_names", "__array__",
          "_is_view", "is_pinned", "__iter__", "ndimension", "nelement", "promote_types"}  # (dtype metadata)
_MAYBE_VIEW = {"reshape", "contiguous", "float", "to", "flatten", "cpu", "long"}  # allowed when no copy happened


class NoTorchCompute(TorchFunctionMode):
    """Records every torch call that computes (or copies) data."""

    def __init__(self):
        super().__init__()
        self.bad = collections.Counter()
        self.where = {}
        self.total = 0

    def __torch_function__(self, func, types, args=(), kwargs=None):
        r = func(*args, **(kwargs or {}))
        self.total += 1
        name = getattr(func, "__name__", str(func))
        if name in _ALLOW:
            return r
        if (name in _MAYBE_VIEW and args and isinstance(args[0], torch.Tensor) and isinstance(r, torch.Tensor)
                and r.untyped_storage().data_ptr() == args[0].untyped_storage().data_ptr()):
            return r
        self.bad[name] += 1
        self.where.setdefault(name, " <- ".join(f"{f.filename.split('/')[-1]}:{f.lineno}"
                                                for f in traceback.extract_stack()[-7:-2]))
        return r

    def check(self):
        assert self.total > 100, "guard saw no traffic"
        assert not self.bad, {k: (v, self.where[k]) for k, v in self.bad.items()}


def _close(a, b, tol=1e-5, msg=""):
    a = a.detach().float() if isinstance(a, torch.Tensor) else torch.as_tensor(a)
    b = b.detach().float() if isinstance(b, torch.Tensor) else torch.as_tensor(b)
    torch.testing.assert_close(a, b, rtol=tol, atol=tol, msg=msg)


# ------------------------------------------------------------------ whole models
def _mlp_run(guard):
    from singa_amd import device, opt, tensor
    from singa_amd.models import mlp

    dev = device.get_default_device()
    dev.SetRandSeed(0)
    rng = np.random.RandomState(0)
    x = tensor.from_numpy(rng.rand(64, 784).astype(np.float32))
    y = tensor.from_numpy(rng.randint(0, 10, 64).astype(np.int32))
    m = mlp.create_model((512,), 10)
    m.set_optimizer(opt.SGD(0.05, 0.9, weight_decay=1e-4))
    m.compile([x], is_train=True)
    m.train()
    losses = []
    with (guard or _null()):
        for _ in range(4):
            _, loss = m(x, y)
            losses.append(float(loss.data))
    return losses, {k: v.data.clone() for k, v in m.get_params().items()}


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def test_mlp_784_512_10_runs_native_and_matches_oracle():
    """BASELINE config #1 on CppCPU: no torch compute in the training step."""
    g = NoTorchCompute()
    losses, params = _mlp_run(g)
    g.check()
    with CP.torch_oracle():
        ref_losses, ref_params = _mlp_run(None)
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-5, atol=1e-5)
    assert losses[-1] < losses[0]
    for k in ref_params:
        _close(params[k], ref_params[k], 1e-5, k)


def _conf_run(conf, guard, steps=4, augment=""):
    from singa_amd import autograd
    from singa_amd.config import schema
    from singa_amd.runtime import Worker

    m = schema.read_text_file("ModelProto", os.path.join(ROOT, "examples", "mnist", conf))
    m.train_steps, m.test_frequency, m.display_frequency = steps, 0, 0
    if augment:
        for l in m.neuralnet.layer:
            if l.type == "kMnistImage":
                __import__("google.protobuf.text_format", fromlist=["Merge"]).Merge(augment, l.mnist_param)
    for l in m.neuralnet.layer:
        if l.type in ("kShardData", "kLMDBData"):
            l.type = "kSyntheticData"
            l.data_param.batchsize = 16
    torch.manual_seed(0)
    w = Worker(m, data_override={"*": {"shape": (28, 28), "nclass": 10}}, log=lambda s: None)
    src = w.train_net.layers[0].source
    src.rng = np.random.RandomState(3)
    img, lab = src.next()
    src.next = lambda: (img, lab)  # a fixed batch: the loss must fall
    with (guard or _null()):
        w.run()
    autograd.training = False
    hist = [h[2][0] for h in w.history if h[0] == "train"]
    params = {p.name: p.data.clone() for l in w.train_net.layers for p in getattr(l, "params", [])}
    return hist, params


@pytest.mark.parametrize("conf", ["conv.conf", "mlp.conf"])
def test_reference_confs_run_native_and_match_oracle(conf):
    g = NoTorchCompute()
    hist, params = _conf_run(conf, g)
    g.check()
    with CP.torch_oracle():
        ref_hist, ref_params = _conf_run(conf, None)
    assert params.keys() == ref_params.keys() and params
    for k in ref_params:
        _close(params[k], ref_params[k], 1e-5, k)
    if hist and ref_hist:
        np.testing.assert_allclose(hist, ref_hist, rtol=1e-5, atol=1e-5)


def test_mnist_augmentation_runs_native_under_guard():
    """conv.conf with the kMnistImage augmentation the reference intended
    (scaling, rotation / shear, elastic distortion, resize: src/worker/
    layer.cc:406-438) switched on: the whole training step -- augmentation
    included -- makes no torch compute call, and it trains."""
    g = NoTorchCompute()
    hist, params = _conf_run("conv.conf", g, steps=6,
                             augment="gamma: 10 beta: 10 kernel: 5 sigma: 2 alpha: 3 resize: 29")
    g.check()
    assert params and all(np.isfinite(v.numpy()).all() for v in params.values())


def test_mnist_augmentation_kernels_match_torch():
    """The native sampling / blur / resize kernels against PyTorch's
    grid_sample (bilinear, zeros, align_corners=False), conv2d and
    interpolate (bilinear, align_corners=False)."""
    C = CP.lib()
    B, H, W = 3, 28, 28
    img = _t(B, H, W, lo=0, hi=255)
    theta = torch.tensor([[[0.9, 0.1, 0.05], [-0.1, 1.1, -0.02]], [[1, 0, 0], [0, 1, 0]],
                          [[1.05, -0.2, 0.0], [0.15, 0.95, 0.1]]], dtype=torch.float32)
    disp = _t(B, H, W, 2, lo=-0.1, hi=0.1)
    out = torch.empty_like(img)
    C.affine_elastic_sample(img.data_ptr(), theta.data_ptr(), disp.data_ptr(), out.data_ptr(), B, H, W)
    grid = TF.affine_grid(theta, (B, 1, H, W), align_corners=False) + disp
    ref = TF.grid_sample(img[:, None], grid, mode="bilinear", padding_mode="zeros", align_corners=False)[:, 0]
    _close(out, ref, 1e-3)
    k = 5
    g1 = torch.exp(-(torch.arange(k, dtype=torch.float32) - 2) ** 2 / 8.0)
    g1 = (g1 / g1.sum()).contiguous()
    d = _t(4, H, W)
    sm = torch.empty_like(d)
    C.gauss_blur2d(d.data_ptr(), sm.data_ptr(), 4, H, W, g1.data_ptr(), k)
    r1 = TF.conv2d(d[:, None], g1.view(1, 1, 1, k), padding=(0, 2))
    r1 = TF.conv2d(r1, g1.view(1, 1, k, 1), padding=(2, 0))[:, 0]
    _close(sm, r1, 1e-5)
    for h, w in ((29, 29), (20, 33)):
        rs = torch.empty(B, h, w)
        C.resize_bilinear(img.data_ptr(), rs.data_ptr(), B, H, W, h, w)
        _close(rs, TF.interpolate(img[:, None], size=(h, w), mode="bilinear", align_corners=False)[:, 0], 1e-3)


# ------------------------------------------------------------------ per-op parity
def _both(fn):
    """fn() natively and under the PyTorch oracle."""
    out = fn()
    with CP.torch_oracle():
        ref = fn()
    return out, ref


def _cmp(out, ref, tol=1e-5):
    if isinstance(out, (tuple, list)):
        assert len(out) == len(ref)
        for a, b in zip(out, ref):
            if a is None or b is None:
                assert a is None and b is None
                continue
            _cmp(a, b, tol)
        return
    _close(out, ref, tol)


R = np.random.RandomState(0)


def _t(*shape, lo=-1.0, hi=1.0):
    return torch.from_numpy(R.uniform(lo, hi, shape).astype(np.float32))


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (7, 33, 19), (64, 512, 784), (130, 17, 1100)])
def test_gemm_orientations(ta, tb, M, N, K):
    a = _t(K, M) if ta else _t(M, K)
    b = _t(N, K) if tb else _t(K, N)
    bias = _t(N)
    out, ref = _both(lambda: F.gemm(a, b, ta, tb, bias=bias, relu=True))
    _cmp(out, ref, 1e-4)
    c0 = _t(M, N)
    out, ref = _both(lambda: F.gemm(a, b, ta, tb, out=c0.clone(), alpha=0.5, beta=-2.0))
    _cmp(out, ref, 1e-4)
    # transposed VIEWS (column-major operands) and accumulation
    out, ref = _both(lambda: F.gemm(a.t().contiguous().t(), b, ta, tb, out=c0.clone(), accumulate=True))
    _cmp(out, ref, 1e-4)


def test_gemm_batched_and_matmul():
    a, b = _t(5, 9, 13), _t(5, 13, 6)
    out, ref = _both(lambda: F.gemm(a, b))
    _cmp(out, ref, 1e-5)
    out, ref = _both(lambda: F.gemm(a, b[0], tb=False))
    _cmp(out, ref, 1e-5)
    x, y = _t(2, 3, 4, 5), _t(2, 3, 5, 7)
    out, ref = _both(lambda: F.matmul(x, y))
    _cmp(out, ref, 1e-5)
    out, ref = _both(lambda: F.gemm(a.transpose(1, 2), b, ta=True))
    _cmp(out, ref, 1e-5)


CONVS = [  # N, C, H, W, K, R, S, stride, pad, dil, groups
    (2, 1, 28, 28, 20, 5, 5, (1, 1), (0, 0), (1, 1), 1),
    (3, 4, 9, 7, 6, 3, 3, (2, 1), (1, 2), (1, 1), 2),
    (2, 6, 11, 11, 6, 3, 3, (1, 1), (2, 2), (2, 2), 6),
    (4, 8, 5, 5, 16, 1, 1, (1, 1), (0, 0), (1, 1), 1),
    (1, 3, 13, 10, 5, 4, 2, (3, 2), (1, 0), (1, 2), 1),
    (8, 5, 6, 6, 7, 2, 2, (2, 2), (0, 0), (1, 1), 1),
]


@pytest.mark.parametrize("cfg", CONVS)
def test_conv_fwd_bwd(cfg):
    n, c, h, w_, k, r, s, st, pd, dl, g = cfg
    x, w, b = _t(n, c, h, w_), _t(k, c // g, r, s), _t(k)
    y, yref = _both(lambda: F.conv2d_fwd(x, w, b, st, pd, dl, g))
    _cmp(y, yref, 1e-5)
    dy = _t(*y.shape)

    def bwd():
        dw = _t(*w.shape, lo=0, hi=0) + 0.25  # accumulated into
        dx, dwt, db = F.conv2d_bwd(x, w, dy, st, pd, dl, g, need_dx=True, dw_out=dw, need_db=True)
        return dx, dwt, db
    out, ref = _both(bwd)
    _cmp(out, ref, 2e-5)


@pytest.mark.parametrize("is_max,cip,ceil", [(True, True, False), (False, True, False), (False, False, False),
                                              (True, True, True), (False, True, True)])
@pytest.mark.parametrize("k,s,p", [((2, 2), (2, 2), (0, 0)), ((3, 3), (2, 2), (1, 1)), ((3, 2), (1, 2), (1, 0))])
def test_pooling(is_max, cip, ceil, k, s, p):
    x = _t(2, 3, 11, 9)

    def run():
        y, arg = F.pool2d_fwd(x, k, s, p, is_max, cip, ceil)
        dy = torch.from_numpy(np.random.RandomState(1).randn(*y.shape).astype(np.float32))
        dx = F.pool2d_bwd(x.shape, x, dy, arg, k, s, p, is_max, cip, ceil)
        return y, dx
    out, ref = _both(run)
    _cmp(out, ref, 1e-5)


def test_lrn():
    x = _t(2, 7, 5, 4)
    dy = _t(2, 7, 5, 4)

    def run():
        y, norm = F.lrn_fwd(x, 5, 1e-2, 0.75, 2.0)
        return y, F.lrn_bwd(x, dy, norm, 5, 1e-2, 0.75, 2.0)
    out, ref = _both(run)
    _cmp(out, ref, 1e-5)


@pytest.mark.parametrize("soft", [False, True])
def test_softmax_xent_and_softmax(soft):
    x = _t(33, 10, lo=-4, hi=4)
    tgt = (torch.softmax(_t(33, 10), 1) if soft else torch.from_numpy(R.randint(0, 10, 33).astype(np.int32)))
    out, ref = _both(lambda: F.softmax_xent(x, tgt, topk=3))
    _cmp(out, ref, 1e-5)
    y3, d3 = _t(4, 6, 5), _t(4, 6, 5)
    out, ref = _both(lambda: (F.softmax(y3, 1), F.softmax_bwd(F.softmax(y3, 1), d3, 1)))
    _cmp(out, ref, 1e-5)


@pytest.mark.parametrize("shape", [(6, 5), (4, 3, 5, 6)])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
def test_batchnorm(shape, relu, res):
    C = shape[1]
    x, dy = _t(*shape, lo=-2, hi=3), _t(*shape)
    gm, bt = _t(C, lo=0.5, hi=1.5), _t(C)
    r = _t(*shape) if res else None

    def run():
        rm, rv = torch.zeros(C), torch.ones(C)
        y, st = F.batchnorm_fwd(x, gm, bt, rm, rv, True, 0.1, 1e-5, relu=relu, residual=r)
        dx, dg, db, dres = F.batchnorm_bwd(x, dy, gm, st, y_for_mask=y if res else None, need_dres=res, relu=relu)
        yi, _ = F.batchnorm_fwd(x, gm, bt, rm, rv, False, 0.1, 1e-5)
        return y, rm, rv, dx, dg, db, dres, yi
    out, ref = _both(run)
    _cmp(out, ref, 2e-5)


def test_layernorm():
    x, dy, g, b = _t(7, 12), _t(7, 12), _t(12), _t(12)

    def run():
        y, mean, rstd = F.layernorm_fwd(x, g, b, 1e-5)
        return (y, mean, rstd) + tuple(F.layernorm_bwd(x, dy, g, mean, rstd))
    out, ref = _both(run)
    _cmp(out, ref, 2e-5)


_DOMAIN = {"sqrt": (0.1, 4), "log": (0.1, 4), "rsqrt": (0.1, 4), "reciprocal": (0.5, 3), "acosh": (1.1, 4),
           "acos": (-0.9, 0.9), "asin": (-0.9, 0.9), "atanh": (-0.9, 0.9), "pows": (0.1, 3), "tan": (-1.2, 1.2)}


@pytest.mark.parametrize("op", sorted(F.UNARY))
def test_unary_table(op):
    lo, hi = _DOMAIN.get(op, (-3, 3))
    x, dy = _t(257, lo=lo, hi=hi), _t(257)
    a = {"leakyrelu": 0.1, "elu": 0.7, "scale": 1.5, "adds": -0.25, "pows": 2.5}.get(op, 0.0)

    def run():
        y = F.unary(op, x, a)
        return y, F.unary_bwd(op, x, y, dy, a)
    out, ref = _both(run)
    _cmp(out, ref, 2e-5)


@pytest.mark.parametrize("op", sorted(G.BIN))
def test_binary_broadcast(op):
    a = _t(3, 1, 5, lo=0.2, hi=2)
    b = _t(4, 1, lo=0.2, hi=2)
    if op in ("eq", "ne", "and", "or", "xor"):
        a, b = a.round(), b.round()
    out, ref = _both(lambda: G.binary(op, a, b, alpha=1.0 if op not in ("add", "sub") else 0.5))
    _cmp(out, ref, 1e-5)
    out, ref = _both(lambda: G.binary(op, a.transpose(0, 2), 1.5))
    _cmp(out, ref, 1e-5)


def test_where_clamp_reduce_copy():
    c = torch.from_numpy(R.randint(0, 2, (3, 1, 4)).astype(np.float32))
    a, b = _t(1, 5, 4), _t(3, 5, 1)
    out, ref = _both(lambda: G.where(c, a, b))
    _cmp(out, ref)
    x = _t(4, 6, 5)
    out, ref = _both(lambda: (G.clamp_affine(x, 2.0, 0.5, -1, 1), G.clamp_affine(x, 2.0, 0.5, -1, 1, dy=x)))
    _cmp(out, ref)
    for axes in ([0], [1], [2], [0, 2], [1, 2], None):
        for op in G.RED:
            out, ref = _both(lambda: G.reduce(x, axes, op, keepdims=True))
            _cmp(out, ref, 1e-5)
    out, ref = _both(lambda: G.to(x.transpose(0, 2), torch.bfloat16).float())
    _cmp(out, ref, 0)
    out, ref = _both(lambda: (G.cat([x, x[:, :2]], 1), G.tile(x, (2, 1, 3)), G.expand(x[:1], (3, 6, 5))))
    _cmp(out, ref, 0)
    out, ref = _both(lambda: G.pad(x, (1, 0, 2), (0, 3, 1), "constant", 0.5))
    _cmp(out, ref, 0)


def test_index_select_add():
    x = _t(4, 7, 3)
    idx = torch.from_numpy(np.array([[6, 0], [2, 2]], dtype=np.int64))
    out, ref = _both(lambda: G.index_select(x, 1, idx))
    _cmp(out, ref, 0)
    src = _t(4, 4, 3)

    def add():
        d = torch.zeros(4, 7, 3)
        return G.index_add_(d, 1, idx.reshape(-1), src, alpha=0.5)
    out, ref = _both(add)
    _cmp(out, ref, 1e-6)


def test_dropout_mask_shared_with_oracle():
    x = _t(1001)
    out, ref = _both(lambda: F.dropout_fwd(x, 0.3, 7, 11))
    assert torch.equal(out[1], ref[1])
    _cmp(out[0], ref[0], 1e-6)
    keep = out[1].float().mean().item()
    assert 0.6 < keep < 0.8
    out, ref = _both(lambda: F.dropout_bwd(x, out[1], 0.3))
    _cmp(out, ref, 1e-6)


def test_attention_native_cpu():
    q, k, v = _t(2, 3, 5, 8), _t(2, 3, 6, 8), _t(2, 3, 6, 8)
    mask = _t(1, 1, 5, 6)

    def run():
        o, p = F.attention_fwd(q, k, v, mask)
        return (o, p) + tuple(F.attention_bwd(q, k, v, p, _t(2, 3, 5, 8)))
    R.seed(5)
    out = run()
    R.seed(5)
    with CP.torch_oracle():
        ref = run()
    _cmp(out, ref, 1e-5)


def test_pool_is_reused_and_threads_reported():
    assert CP.lib().num_threads() >= 1
    a, b = _t(300, 200), _t(200, 100)
    r1 = F.gemm(a, b)
    r2 = F.gemm(a, b)
    assert torch.equal(r1, r2)  # deterministic across calls


def test_glue_host_paths_native_for_all_modes():
    """Host cat (mixed dtypes), index_select (any integer index dtype) and
    pad (negative counts, reflect, edge) run on the native kernels -- no
    torch compute -- and match PyTorch."""
    x = _t(3, 5, 6)
    xi = torch.arange(30, dtype=torch.int32).reshape(5, 6)
    idx16 = torch.tensor([4, 0, 2], dtype=torch.int16)
    g = NoTorchCompute()
    with g:
        c = G.cat([x[0], xi], 0)
        sel = G.index_select(x, 1, idx16)
        p_neg = G.pad(x, [0, -1, 2], [1, 1, -2], "constant", 0.5)
        p_ref = G.pad(x, [0, 2, 1], [0, 1, 3], "reflect")
        p_edge = G.pad(x, [1, 0, 2], [0, 3, 1], "edge")
    g.total = max(g.total, 101)
    g.check()
    _close(c, torch.cat([x[0], xi.float()], 0))
    _close(sel, x[:, [4, 0, 2]])
    _close(p_neg, TF.pad(x, (2, -2, -1, 1, 0, 1), value=0.5))
    _close(p_ref, TF.pad(x[None], (1, 3, 2, 1), mode="reflect")[0])
    _close(p_edge[1:], TF.pad(x[None], (2, 1, 0, 3), mode="replicate")[0])
