"""Glue kernels (csrc/kernels/glue.hip, new elementwise ops) against plain
PyTorch fp32 CPU references, plus autograd-level forward/backward of every
glue operator on the GPU vs. the same graph on the CPU."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _r(*shape, seed=0, dtype=torch.float32):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)).to(dtype)


@pytest.mark.parametrize("dt_in,dt_out", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                          (torch.bfloat16, torch.float32), (torch.int64, torch.float32),
                                          (torch.float32, torch.int32)])
def test_copy_nd_permute_cast(gpu, dt_in, dt_out):
    from singa_amd.ops import glue as G
    x = (_r(3, 5, 7, 4, seed=1) * 10).to(dt_in)
    xg = x.to(gpu)
    y = G.to(G.contiguous(xg.permute(2, 0, 3, 1)), dt_out)
    ref = x.permute(2, 0, 3, 1).contiguous().to(dt_out)
    assert y.dtype == dt_out and torch.equal(y.cpu(), ref)
    cl = G.to(xg.to(torch.float32) if dt_in == torch.int64 else xg, memory_format=torch.channels_last)
    assert cl.is_contiguous(memory_format=torch.channels_last) and torch.equal(cl.cpu().float(), x.float())


def test_copy_broadcast_tile_expand(gpu):
    from singa_amd.ops import glue as G
    x = _r(2, 1, 3, seed=2)
    assert torch.equal(G.expand(x.to(gpu), (4, 2, 5, 3)).cpu(), x.expand(4, 2, 5, 3))
    assert torch.equal(G.tile(x.to(gpu), [2, 3, 1]).cpu(), x.repeat(2, 3, 1))
    g = _r(4, 3, 3, seed=3)
    assert rel_err(G.tile_backward(g.to(gpu), [2, 3, 1], (2, 1, 3)), g.reshape(2, 2, 3, 1, 1, 3).sum((0, 2, 4))) < 1e-6


@pytest.mark.parametrize("op", ["add", "sub", "mul", "div", "pow", "max", "min", "lt", "ge", "eq", "and", "xor"])
def test_binary_broadcast(gpu, op):
    from singa_amd.ops import glue as G
    a = _r(4, 1, 6, seed=4).abs() + 0.5
    b = _r(3, 1, seed=5).abs() + 0.5
    if op in ("eq",):
        b = a[0, :, :3].reshape(3, 1).clone()
    y = G.binary(op, a.to(gpu), b.to(gpu))
    ref = G.binary(op, a, b)  # CPU reference path
    assert y.shape == ref.shape and rel_err(y, ref) < 1e-6
    yb = G.binary(op, a.to(gpu).bfloat16(), b.to(gpu).bfloat16())
    assert yb.dtype == torch.bfloat16 and rel_err(yb, ref) < 2e-2


def test_where_clamp(gpu):
    from singa_amd.ops import glue as G
    c = (_r(5, 1, seed=6) > 0)
    a, b = _r(5, 4, seed=7), _r(1, 4, seed=8)
    assert torch.equal(G.where(c.to(gpu), a.to(gpu), b.to(gpu)).cpu(), torch.where(c, a, b))
    x = _r(1000, seed=9)
    assert torch.allclose(G.clamp_affine(x.to(gpu), 0.2, 0.5, 0.0, 1.0).cpu(), torch.clamp(0.2 * x + 0.5, 0, 1),
                          rtol=1e-6, atol=1e-7)  # (fused multiply-add on the GPU)
    d = _r(1000, seed=10)
    gd = G.clamp_affine(x.to(gpu), 0.2, 0.5, 0.0, 1.0, dy=d.to(gpu)).cpu()
    z = 0.2 * x + 0.5
    assert torch.allclose(gd, d * 0.2 * ((z > 0) & (z < 1)).float())


@pytest.mark.parametrize("axes", [None, [0], [1], [2], [0, 2], [1, 2], [0, 1, 2]])
@pytest.mark.parametrize("op", ["sum", "mean", "max", "min", "sumsq"])
def test_reduce(gpu, axes, op):
    from singa_amd.ops import glue as G
    x = _r(6, 33, 10, seed=11)
    y = G.reduce(x.to(gpu), axes, op, keepdims=True)
    ref = G.reduce(x, axes, op, keepdims=True)
    assert y.shape == ref.shape and rel_err(y, ref) < 1e-5


def test_reduce_long_row_split(gpu):
    from singa_amd.ops import glue as G
    x = _r(3, 300000, seed=12)
    assert rel_err(G.reduce(x.to(gpu), [1], "sum"), x.double().sum(1)) < 1e-5
    assert rel_err(G.reduce(x.to(gpu).bfloat16(), None, "mean", out_dtype=torch.float32),
                   x.bfloat16().double().mean()) < 1e-4


def test_index_select_add(gpu):
    from singa_amd.ops import glue as G
    W = _r(1000, 768, seed=13).bfloat16()
    idx = torch.randint(0, 1000, (4, 128), generator=torch.Generator().manual_seed(1))
    y = G.index_select(W.to(gpu), 0, idx.to(gpu))
    assert torch.equal(y.cpu(), W[idx])
    x = _r(5, 7, 3, seed=14)
    i2 = torch.tensor([[6, 0], [2, -1]])
    assert torch.equal(G.index_select(x.to(gpu), 1, i2.to(gpu)).cpu(), x[:, i2.remainder(7)])
    dW = torch.zeros(1000, 768)
    dy = _r(4 * 128, 768, seed=15)
    G.index_add_(dW_g := dW.to(gpu), 0, idx.reshape(-1).to(gpu), dy.to(gpu))
    assert rel_err(dW_g, torch.zeros(1000, 768).index_add_(0, idx.reshape(-1), dy)) < 1e-6


def test_gather_scatter_elements(gpu):
    from singa_amd.ops import glue as G
    x = _r(4, 9, 5, seed=16)
    idx = torch.randint(0, 9, (4, 3, 5), generator=torch.Generator().manual_seed(2))
    assert torch.equal(G.gather_elements(x.to(gpu), 1, idx.to(gpu)).cpu(), torch.gather(x, 1, idx))
    u = _r(4, 3, 5, seed=17)
    idx_u = torch.stack([torch.randperm(9, generator=torch.Generator().manual_seed(i))[:3] for i in range(20)]) \
        .reshape(4, 5, 3).permute(0, 2, 1).contiguous()
    ref = x.scatter(1, idx_u, u)
    assert torch.equal(G.scatter_elements(x.to(gpu), 1, idx_u.to(gpu), u.to(gpu)).cpu(), ref)


@pytest.mark.parametrize("mode", ["constant", "reflect", "edge"])
def test_pad_and_backward(gpu, mode):
    from singa_amd.ops import glue as G
    x = _r(2, 3, 5, 6, seed=18)
    before, after = [0, 1, 2, 3], [1, 0, 3, 2]
    y = G.pad(x.to(gpu), before, after, mode, 1.5)
    ref = G.pad(x, before, after, mode, 1.5)
    assert torch.equal(y.cpu(), ref)
    dy = _r(*ref.shape, seed=19)
    assert rel_err(G.pad_backward(dy.to(gpu), x.shape, before, mode), G.pad_backward(dy, x.shape, before, mode)) < 1e-6


@pytest.mark.parametrize("op", ["erf", "cos", "sin", "tan", "cosh", "sinh", "atan", "asinh", "ceil", "floor",
                                "round", "softsign", "rsqrt", "scale", "adds", "pows"])
def test_new_unary_fwd_bwd(gpu, op):
    from singa_amd.ops import functional as F
    x = _r(4099, seed=20) * 0.9
    if op in ("rsqrt", "pows"):
        x = x.abs() + 0.1
    a = {"scale": 1.7, "adds": -0.3, "pows": 2.5}.get(op, 0.0)
    y = F.unary(op, x.to(gpu), a)
    ref = F.unary(op, x, a)
    assert rel_err(y, ref) < 1e-5
    dy = _r(4099, seed=21)
    g = F.unary_bwd(op, x.to(gpu), y, dy.to(gpu), a)
    gref = F.unary_bwd(op, x, ref, dy, a)
    assert rel_err(g, gref) < 1e-5


def _graph(dev, fn, *arrays):
    """Run fn on singa tensors on `dev`; returns (outputs, input grads)."""
    from singa_amd import autograd, tensor
    ts = []
    for a in arrays:
        t = tensor.from_numpy(a).to_device(dev)
        t.requires_grad = t.stores_grad = a.dtype == np.float32
        ts.append(t)
    autograd.training = True
    try:
        y = fn(*ts)
        loss = autograd.reduce_sum(autograd.mul(y, y))
        grads = {id(p): g for p, g in autograd.backward(loss)}
    finally:
        autograd.training = False
    return y.data.float().cpu(), [grads[id(t)].data.float().cpu() if id(t) in grads else None for t in ts]


GLUE_CASES = {
    "transpose": (lambda A, x: A.transpose(x, (2, 0, 1)), [(3, 4, 5)]),
    "cat_split": (lambda A, x, y: A.split(A.cat([x, y], 1), 1, [2, 5])[1], [(3, 4), (3, 3)]),
    "slice": (lambda A, x: A.slice(x, [1, 0], [3, 4], [0, 2], [1, 2]), [(4, 3, 5)]),
    "gather": (lambda A, x: A.gather(x, 1, [3, 0, 3]), [(2, 5, 3)]),
    "tile_expand": (lambda A, x: A.add(A.tile(x, [2, 1]), A.expand(x, (2, 3))), [(1, 3)]),
    "pad_reflect": (lambda A, x: A.pad(x, "reflect", [1, 2, 1, 0]), [(4, 5)]),
    "clip_where": (lambda A, x, y: A.where(A.clip(x, -0.5, 0.5), y, np.array([[1], [0], [1]], bool)),
                   [(3, 4), (3, 4)]),
    "reduce": (lambda A, x: A.add(A.reduce_mean(x, [1], 1), A.reduce_sum(x, [0, 2], 1)), [(3, 4, 5)]),
    "nary": (lambda A, x, y: A.add(A.max(x, y), A.mean(x, y)), [(3, 4), (1, 4)]),
    "arith": (lambda A, x, y: A.div(A.sub(A.mul(x, y), y), A.add(A.abs(y), A.abs(y))), [(3, 4), (4,)]),
    "math": (lambda A, x: A.add(A.erf(A.sin(x)), A.hardsigmoid(A.atan(x))), [(5, 6)]),
    "prelu": (lambda A, x, s: A.prelu(x, s), [(4, 3), (3,)]),
    "space": (lambda A, x: A.depth_to_space(A.space_to_depth(x, 2), 2, "CRD"), [(2, 4, 4, 6)]),
    "upsample": (lambda A, x: A.upsample(x, "nearest", [1, 1, 2, 3]), [(1, 2, 3, 2)]),
    "gemm": (lambda A, x, w, c: A.gemm(x, w, c, 0.5, 2.0, 0, 1), [(5, 7), (3, 7), (1, 3)]),
}


@pytest.mark.parametrize("name", sorted(GLUE_CASES))
def test_autograd_glue_gpu_vs_cpu(gpu, name):
    from singa_amd import autograd as A
    from singa_amd import device
    fn, shapes = GLUE_CASES[name]
    rng = np.random.RandomState(0)
    arrays = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    yc, gc = _graph(device.get_default_device(), lambda *t: fn(A, *t), *arrays)
    yg, gg = _graph(device.create_rocm_gpu(), lambda *t: fn(A, *t), *arrays)
    assert yg.shape == yc.shape and rel_err(yg, yc) < 1e-5
    for a, b in zip(gg, gc):
        if b is not None:
            assert a is not None and rel_err(a, b) < 1e-5
