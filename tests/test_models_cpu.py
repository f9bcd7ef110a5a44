"""Model zoo on CPU: every family trains a few steps on a fixed batch; the
attention operator passes a finite-difference check."""
import numpy as np
import pytest
import torch

from singa_amd import autograd, device, opt, tensor
from singa_amd.tensor import Tensor


def _train(m, x, y, steps=6, lr=0.01, **kw):
    device.get_default_device().SetRandSeed(0)
    m.set_optimizer(opt.SGD(lr, 0.9))
    m.compile([x], is_train=True)
    ls = []
    for _ in range(steps):
        _, l = m(x, y, **kw)
        ls.append(float(l.data))
    return ls


def _img(n, c, h, w, k=10, seed=0):
    rng = np.random.RandomState(seed)
    return (tensor.from_numpy(rng.randn(n, c, h, w).astype(np.float32)),
            tensor.from_numpy(rng.randint(0, k, n).astype(np.int32)))


@pytest.mark.parametrize("name", ["mlp", "deep_big_simple", "cnn", "alexnet_small", "vgg11_small", "resnet18"])
def test_model_trains(name):
    from singa_amd.models import alexnet, cnn, mlp, resnet, vgg

    if name == "mlp":
        m, (x, y) = mlp.MLP((64,)), _img(8, 1, 8, 8)
    elif name == "deep_big_simple":
        m, (x, y) = mlp.deep_big_simple(), _img(4, 1, 28, 28)
    elif name == "cnn":
        m, (x, y) = cnn.CNN(), _img(4, 1, 28, 28)
    elif name == "alexnet_small":
        m, (x, y) = alexnet.AlexNet(10, small=True), _img(4, 3, 32, 32)
    elif name == "vgg11_small":
        m, (x, y) = vgg.VGG(11, 10, small=True), _img(2, 3, 32, 32)
    else:
        m, (x, y) = resnet.resnet18(num_classes=10), _img(2, 3, 32, 32)
    ls = _train(m, x, y, lr=0.005 if name != "mlp" else 0.05)
    assert all(np.isfinite(ls)) and ls[-1] < ls[0], ls


def test_bert_tiny_trains():
    from singa_amd.models import bert

    rng = np.random.RandomState(0)
    ids = tensor.from_numpy(rng.randint(0, 1000, (4, 16)).astype(np.int64))
    y = tensor.from_numpy(rng.randint(0, 2, 4).astype(np.int32))
    mask = torch.ones(4, 16)
    mask[:, 12:] = 0
    ls = _train(bert.bert_tiny(dropout=0.0), ids, y, lr=0.01, mask=Tensor(data=mask, requires_grad=False))
    assert all(np.isfinite(ls)) and ls[-1] < ls[0], ls


def test_attention_grad_fd():
    rng = np.random.RandomState(1)
    q, k, v = (Tensor(data=torch.tensor(rng.randn(2, 3, 4), dtype=torch.float32)) for _ in range(3))
    mask = torch.zeros(1, 3, 3)
    mask[..., 2] = -1e4
    autograd.training = True
    for t in (q, k, v):
        t.requires_grad = t.stores_grad = True

    def f(q, k, v):
        o = autograd.attention(q, k, v, Tensor(data=mask, requires_grad=False))
        return autograd.reduce_sum(autograd.mul(o, o), None)

    y = f(q, k, v)
    g = {id(p): d.data.clone() for p, d in autograd.backward(y)}
    eps = 1e-3
    for t in (q, k, v):
        flat = t.data.view(-1)
        for i in range(0, flat.numel(), 5):
            old = float(flat[i])
            flat[i] = old + eps
            fp = float(f(q, k, v).data)
            flat[i] = old - eps
            fm = float(f(q, k, v).data)
            flat[i] = old
            num = (fp - fm) / (2 * eps)
            assert abs(num - float(g[id(t)].view(-1)[i])) < 2e-2 * max(1.0, abs(num)), (num, g[id(t)].view(-1)[i])
    autograd.training = False


def test_sublayers_in_lists_filled_after_assignment():
    """``self.blocks = []`` followed by appends (VGG) must still expose every
    parameter to get_params / the optimiser."""
    from singa_amd.models import vgg

    m = vgg.create_model(11, num_classes=10)
    x = tensor.from_numpy(np.random.RandomState(0).randn(2, 3, 32, 32).astype(np.float32))
    m.compile([x], is_train=False)
    names = list(m.get_params())
    assert sum(n.startswith("convs.") for n in names) == 8  # 8 conv weights (no bias with BN)
    assert sum(n.startswith("bns.") for n in names) == 16  # gamma, beta
    assert any(k.startswith("bns.") and "mean" in k for k in m.get_states())
