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


def test_paired_stem_index_maps_cpu():
    """The paired-tap stem identity the GPU stem relies on: a 7x7/2/p3 conv
    over C <= 3 channels equals a 7x4 conv (horizontal dilation 2, pad (3, 2))
    over "pair" pixels {x(w-1, :3), x(w, :3), 0, 0} of width W+1, with the
    weight re-laid by ``_pair_maps``; and its weight gradient maps back."""
    import torch.nn.functional as TF

    from singa_amd.models.resnet import _pair_maps

    torch.manual_seed(0)
    for (H, W, C) in [(16, 16, 3), (15, 13, 3), (12, 10, 1)]:
        K = 5
        x = torch.randn(2, C, H, W, dtype=torch.float64)
        w = torch.randn(K, C, 7, 7, dtype=torch.float64, requires_grad=True)
        ref = TF.conv2d(x, w, stride=2, padding=3)
        xp = torch.zeros(2, 8, H, W + 1, dtype=torch.float64)
        xp[:, :C, :, 1:] = x
        xp[:, 3:3 + C, :, :W] = x
        fwd, bwd = _pair_maps(K, C, "cpu")
        wk = w.detach().permute(0, 2, 3, 1).reshape(-1)
        wp = torch.cat([wk, wk.new_zeros(1)])[fwd].view(K, 7, 4, 8).permute(0, 3, 1, 2).contiguous()
        wp.requires_grad_(True)
        # the GPU kernel takes Ho/Wo explicitly and zero-fills every out-of-range tap:
        # pad generously, then keep the reference's output extent
        y = TF.conv2d(TF.pad(xp, (2, 4, 3, 3)), wp, stride=2, dilation=(1, 2))[..., :ref.shape[2], :ref.shape[3]]
        assert y.shape == ref.shape
        assert torch.allclose(y, ref, atol=1e-9)
        dy = torch.randn_like(ref)
        (ref * dy).sum().backward()
        (y * dy).sum().backward()
        dwp = wp.grad.permute(0, 2, 3, 1).reshape(-1)  # [K][7][4][8] flat
        dw = dwp[bwd].view(K, 7, 7, C).permute(0, 3, 1, 2)
        assert torch.allclose(dw, w.grad, atol=1e-9)
