"""CPU tests of the core API: tensor, autograd (finite-difference checks),
layers, optimisers, model graph/ckpt plumbing, native host runtime."""
import os

import numpy as np
import pytest
import torch

from singa_amd import autograd, device, layer, model, opt, tensor
from singa_amd.tensor import Tensor


def fd_check(fn, inputs, eps=1e-3, tol=2e-2):
    """Finite-difference gradient check of a scalar-valued fn of Tensors."""
    autograd.training = True
    for x in inputs:
        x.requires_grad = True
        x.stores_grad = True
    y = fn(*inputs)
    grads = {id(p): g.data.clone() for p, g in autograd.backward(y)}
    for x in inputs:
        base = x.data.clone()
        flat = x.data.view(-1)
        num = torch.zeros_like(flat)
        for i in range(min(flat.numel(), 12)):
            flat[i] = base.view(-1)[i] + eps
            fp = float(fn(*inputs).data)
            flat[i] = base.view(-1)[i] - eps
            fm = float(fn(*inputs).data)
            flat[i] = base.view(-1)[i]
            num[i] = (fp - fm) / (2 * eps)
        ana = grads[id(x)].reshape(-1)[:12]
        assert torch.allclose(ana, num[:12], rtol=tol, atol=tol), (ana, num[:12])
    autograd.training = False


def T(a):
    return Tensor(data=torch.as_tensor(np.asarray(a, dtype=np.float32)))


def test_tensor_api():
    t = tensor.from_numpy(np.arange(6, dtype=np.float32).reshape(2, 3))
    assert t.shape == (2, 3) and t.ndim() == 2 and t.size() == 6
    assert np.allclose(tensor.to_numpy(t.T()), np.arange(6).reshape(2, 3).T)
    u = t + 1
    assert np.allclose(tensor.to_numpy(u), np.arange(6).reshape(2, 3) + 1)
    m = tensor.mult(t, t.T())
    assert m.shape == (2, 2)
    z = tensor.zeros((3,))
    z.set_value(2.0)
    assert tensor.sum(z) == 6.0
    r = tensor.Tensor((1000,))
    r.gaussian(1.0, 0.5)
    assert abs(tensor.average(r) - 1.0) < 0.1
    c = tensor.concatenate([t, t], 0)
    assert c.shape == (4, 3)


@pytest.mark.parametrize("op", ["relu", "sigmoid", "tanh", "stanh", "gelu", "softplus", "exp"])
def test_unary_grads(op):
    x = T(np.random.RandomState(0).randn(3, 4) * 0.8 + 0.05)
    f = getattr(autograd, op)
    fd_check(lambda a: autograd.reduce_sum(autograd.mul(f(a), f(a)), None), [x])


def test_linear_conv_bn_pool_grads():
    rng = np.random.RandomState(1)
    x = T(rng.randn(2, 3, 6, 6))
    w = T(rng.randn(4, 3, 3, 3) * 0.3)
    g = T(rng.rand(4) + 0.5)
    b = T(rng.randn(4))
    rm, rv = torch.zeros(4), torch.ones(4)

    def f(x, w, g, b):
        y = autograd.Conv2d((1, 1), (1, 1))(x, w)
        y = autograd.BatchNorm2d(rm, rv, relu=True)(y, g, b)
        y = autograd.Pooling2d((2, 2), (2, 2), is_max=False)(y)
        y = autograd.flatten(y)
        return autograd.reduce_sum(autograd.mul(y, y), None)
    fd_check(f, [x, w, g, b], eps=1e-2, tol=5e-2)


def test_softmax_xent_grad():
    rng = np.random.RandomState(2)
    x = T(rng.randn(5, 7))
    t = Tensor(data=torch.tensor([1, 2, 3, 0, 6]), requires_grad=False)
    fd_check(lambda a: autograd.softmax_cross_entropy(a, t), [x])


def test_matmul_and_linear():
    rng = np.random.RandomState(3)
    a, bm = T(rng.randn(4, 5)), T(rng.randn(5, 3))
    fd_check(lambda a, b: autograd.reduce_sum(autograd.mul(autograd.matmul(a, b), autograd.matmul(a, b)), None),
             [a, bm])
    bias = T(rng.randn(3))
    fd_check(lambda a, b, c: autograd.reduce_sum(autograd.square(autograd.linear(a, b, c)), None), [a, bm, bias])


def test_multi_output_split_grad():
    x = T(np.random.RandomState(4).randn(4, 6))

    def f(a):
        p, q = autograd.split(a, 1, [2, 4])
        return autograd.add(autograd.reduce_sum(autograd.square(p), None),
                            autograd.reduce_sum(autograd.mul(q, q), None))
    fd_check(f, [x])


class MLP(model.Model):
    def __init__(self):
        super().__init__()
        self.l1 = layer.Linear(64)
        self.act = layer.ReLU()
        self.l2 = layer.Linear(10)
        self.loss = layer.SoftMaxCrossEntropy()

    def forward(self, x):
        return self.l2(self.act(self.l1(x)))

    def train_one_batch(self, x, y):
        out = self.forward(x)
        l = self.loss(out, y)
        self.optimizer(l)
        return out, l


@pytest.mark.parametrize("O", [lambda: opt.SGD(0.1, 0.9), lambda: opt.Adam(1e-2), lambda: opt.AdaGrad(0.1),
                               lambda: opt.RMSProp(0.01), lambda: opt.RefSGD(0.1, 0.9)])
def test_mlp_trains(O):
    rng = np.random.RandomState(0)
    X = rng.randn(32, 20).astype(np.float32)
    Y = rng.randint(0, 10, 32).astype(np.int32)
    m = MLP()
    m.set_optimizer(O())
    tx, ty = tensor.from_numpy(X), tensor.from_numpy(Y)
    m.compile([tx], is_train=True)
    first = None
    for _ in range(60):
        _, l = m(tx, ty)
        first = first if first is not None else float(l.data)
    assert float(l.data) < first * 0.5


def test_checkpoint_roundtrip(tmp_path):
    rng = np.random.RandomState(0)
    X = rng.randn(8, 20).astype(np.float32)
    Y = rng.randint(0, 10, 8).astype(np.int32)
    m = MLP()
    m.set_optimizer(opt.SGD(0.1, 0.9))
    tx, ty = tensor.from_numpy(X), tensor.from_numpy(Y)
    m.compile([tx], is_train=True)
    for _ in range(3):
        m(tx, ty)
    f = str(tmp_path / "ck.zip")
    m.save_states(f, {"epoch": 3, "note": "x"})
    m2 = MLP()
    m2.set_optimizer(opt.SGD(0.1, 0.9))
    m2.compile([tx], is_train=True)
    aux = m2.load_states(f)
    assert aux["epoch"] == 3
    for (k, a), (k2, b) in zip(m.get_states().items(), m2.get_states().items()):
        assert k == k2 and torch.allclose(a.data, b.data)
    assert m2.optimizer.step_counter == 3
    _, l1 = m(tx, ty)
    _, l2 = m2(tx, ty)
    assert abs(float(l1.data) - float(l2.data)) < 1e-5  # resume reproduces the loss


@pytest.mark.parametrize("kind", [lambda: opt.SGD(0.1, 0.9), lambda: opt.Adam(1e-3)])
@pytest.mark.parametrize("src_cl,dst_cl", [(True, False), (False, True)])
def test_optimizer_state_portable_across_layouts(kind, src_cl, dst_cl):
    """Optimizer slots are exported per parameter in the LOGICAL layout, so a
    checkpoint written by the GPU store (conv weights KRSC in the flat
    buffer) restores correctly into the CPU store (KCRS) and vice versa.  A
    raw flat copy would scramble conv momentum with no error."""
    rng = np.random.RandomState(0)
    shapes = [(6, 3, 3, 3), (6,), (4, 6, 1, 1), (10, 24)]

    def params():
        return [Tensor(data=torch.as_tensor(rng.randn(*s).astype(np.float32)), requires_grad=True) for s in shapes]

    a, b = kind(), kind()
    a.attach(params(), channels_last=src_cl)
    b.attach(params(), channels_last=dst_cl)
    refs = {}
    for k in ("s1", "s2"):
        flat = getattr(a.store, k)
        if flat is None:
            continue
        refs[k] = [torch.as_tensor(rng.randn(*v.shape).astype(np.float32)) for v in a.store.slot_views(flat)]
        for v, r in zip(a.store.slot_views(flat), refs[k]):
            v.copy_(r)
    a.step_counter = 7
    st = a.get_states()
    b.set_states(st)
    assert b.step_counter == 7
    for k, rs in refs.items():
        for v, r in zip(b.store.slot_views(getattr(b.store, k)), rs):
            assert torch.equal(v, r)
        # the flat buffers differ (that is exactly why a flat copy is wrong)
        assert not torch.equal(getattr(a.store, k), getattr(b.store, k))


def test_native_core_graph_and_shard(tmp_path):
    from singa_amd import _core
    g = _core.Graph()
    for a, b in [("data", "conv1"), ("conv1", "pool1"), ("pool1", "ip1"), ("label", "loss"), ("ip1", "loss")]:
        g.add_edge(a, b)
    order = g.sort()
    assert order.index("conv1") < order.index("pool1") < order.index("ip1") < order.index("loss")
    assert '"directed":1' in g.to_json([0] * 6)
    folder = str(tmp_path / "shard")
    s = _core.Shard(folder, _core.kCreate)
    for i in range(5):
        rec = _core.encode_record([1, 2, 2], i % 10, bytes([i, 1, 2, 255]), [])
        assert s.insert(f"k{i}".encode(), rec)
    assert not s.insert(b"k0", b"dup")
    s.flush()
    assert s.count() == 5
    del s
    r = _core.Shard(folder, _core.kRead)
    k, v = r.next()
    d = _core.decode_record(v)
    assert k == b"k0" and d["shape"] == [1, 2, 2] and d["pixel"] == bytes([0, 1, 2, 255])
    n = 1
    while r.next() is not None:
        n += 1
    assert n == 5
    r.seek_to_first()
    assert r.next()[0] == b"k0"


@pytest.mark.parametrize("k,s,p", [(3, 2, 0), (3, 2, 1), (3, 1, 1), (2, 2, 0)])
def test_cpu_maxpool_backward_overlapping_windows(k, s, p):
    """Overlapping max-pool windows (AlexNet 3x3/2) route several outputs'
    gradients to one input: they must accumulate, not overwrite."""
    import torch.nn.functional as TF
    from singa_amd.ops import functional as F

    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 4, 11, 13, generator=g)
    xr = x.clone().requires_grad_(True)
    yr = TF.max_pool2d(xr, k, s, p)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    y, arg = F.pool2d_fwd(x, (k, k), (s, s), (p, p), True)
    dx = F.pool2d_bwd(x.shape, x, dy, arg, (k, k), (s, s), (p, p), True)
    assert torch.allclose(y, yr.detach()) and torch.allclose(dx, xr.grad, atol=1e-6)
