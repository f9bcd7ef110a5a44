"""Generic MFMA GEMM / convolution kernels (csrc/kernels/ggemm.hip) against
plain PyTorch CPU references: fp32 operands must match an fp32 reference to
1e-5 WITHOUT any bf16 rounding of the inputs (exact-f32 MFMA), bf16 operands
a reference on the bf16-rounded inputs."""
import numpy as np
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _rand(*shape, seed=0, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g).to(dtype)


@pytest.mark.parametrize("M,N,K", [(1, 10, 784), (1024, 2500, 784), (37, 53, 91), (128, 128, 128), (5, 3, 1),
                                   (300, 7, 2000), (64, 1000, 500)])
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_fp32_gemm_exact(gpu, M, N, K, ta, tb):
    from singa_amd.ops import functional as F
    A = _rand(K, M, seed=1) if ta else _rand(M, K, seed=1)
    B = _rand(N, K, seed=2) if tb else _rand(K, N, seed=2)
    c = F.gemm(A.to(gpu), B.to(gpu), ta=ta, tb=tb, out_dtype=torch.float32)
    ref = (A.double().t() if ta else A.double()) @ (B.double().t() if tb else B.double())
    assert rel_err(c, ref) < 1e-5


def test_fp32_gemm_bias_relu_beta_batched(gpu):
    from singa_amd.ops import functional as F
    a, b = _rand(3, 45, 70, seed=3), _rand(3, 70, 33, seed=4)
    bias = _rand(33, seed=5)
    y = F.matmul(a.to(gpu), b.to(gpu), out_dtype=torch.float32, bias=bias.to(gpu), relu=True)
    ref = torch.relu(a.double() @ b.double() + bias.double())
    assert rel_err(y, ref) < 1e-5
    out = _rand(45, 33, seed=6)
    o = out.to(gpu)
    F.gemm(a[0].to(gpu), b[0].to(gpu), out=o, alpha=0.5, beta=2.0)
    assert rel_err(o, 0.5 * (a[0].double() @ b[0].double()) + 2 * out.double()) < 1e-5


def test_fp32_gemm_transposed_views_and_accumulate(gpu):
    from singa_amd.ops import functional as F
    x, dy = _rand(513, 784, seed=7), _rand(513, 250, seed=8)
    acc = _rand(784, 250, seed=9)
    g = acc.to(gpu)
    F.gemm_tn_acc(x.to(gpu), dy.to(gpu), g)  # split-K atomics
    assert rel_err(g, acc.double() + x.double().t() @ dy.double()) < 1e-5
    xt = x.to(gpu).t()  # column-major view: no copy
    c = F.gemm(xt, dy.to(gpu), out_dtype=torch.float32)
    assert rel_err(c, x.double().t() @ dy.double()) < 1e-5


@pytest.mark.parametrize("M,N,K", [(37, 53, 91), (100, 10, 30), (257, 129, 67)])
def test_bf16_ragged_gemm(gpu, M, N, K):
    from singa_amd.ops import functional as F
    A, B = _rand(M, K, seed=10, dtype=torch.bfloat16), _rand(K, N, seed=11, dtype=torch.bfloat16)
    c = F.matmul(A.to(gpu), B.to(gpu), out_dtype=torch.float32)
    assert rel_err(c, A.double() @ B.double()) < 1e-5
    cb = F.matmul(A.to(gpu), B.to(gpu))
    assert cb.dtype == torch.bfloat16 and rel_err(cb, A.double() @ B.double()) < 1e-2


CONVS = [  # N, C, H, W, K, R, S, stride, pad, dil, groups
    (4, 1, 28, 28, 20, 5, 5, 1, 0, 1, 1),     # LeNet conv1 (C = 1)
    (4, 20, 12, 12, 50, 5, 5, 1, 0, 1, 1),    # LeNet conv2
    (2, 6, 15, 17, 12, 3, 3, 2, 1, 1, 3),     # grouped, ragged, stride 2
    (2, 8, 14, 14, 8, 3, 3, 1, 2, 2, 8),      # depthwise, dilated
    (2, 16, 9, 9, 24, 3, 3, 3, 1, 1, 2),      # stride 3
    (2, 5, 11, 10, 7, 1, 1, 1, 0, 1, 1),      # 1x1 ragged
    (2, 12, 10, 10, 16, 3, 5, (2, 1), (0, 2), (1, 2), 4),
]


def _pair(v):
    return v if isinstance(v, tuple) else (v, v)


@pytest.mark.parametrize("cfg", CONVS)
def test_fp32_conv_fwd_bwd_exact(gpu, cfg):
    from singa_amd.ops import functional as F
    Nn, C, H, W, K, R, S, st, pd, dl, g = cfg
    st, pd, dl = _pair(st), _pair(pd), _pair(dl)
    x = _rand(Nn, C, H, W, seed=20)
    w = _rand(K, C // g, R, S, seed=21) * 0.2
    b = _rand(K, seed=22)
    y = F.conv2d_fwd(x.to(gpu), w.to(gpu), b.to(gpu), st, pd, dl, g, out_dtype=torch.float32)
    xd = x.double().requires_grad_(True)
    wd = w.double().requires_grad_(True)
    ref = TF.conv2d(xd, wd, b.double(), st, pd, dl, g)
    assert y.dtype == torch.float32 and rel_err(y, ref) < 1e-5
    dy = _rand(*ref.shape, seed=23)
    gx, gw = torch.autograd.grad(ref, [xd, wd], dy.double())
    dw = torch.zeros(K, C // g, R, S, device=gpu).contiguous(memory_format=torch.channels_last)
    dx, dwt, db = F.conv2d_bwd(x.to(gpu), w.to(gpu), dy.to(gpu), st, pd, dl, g, need_dx=True, dw_out=dw,
                               need_db=True)
    assert rel_err(dx, gx) < 1e-5
    assert dwt is dw and rel_err(dw, gw) < 1e-5
    assert rel_err(db, dy.double().sum((0, 2, 3))) < 1e-5


def test_bf16_grouped_conv(gpu):
    from singa_amd.ops import functional as F
    x = _rand(4, 32, 14, 14, seed=30, dtype=torch.bfloat16)
    w = (_rand(64, 8, 3, 3, seed=31) * 0.2).to(torch.bfloat16)
    y = F.conv2d_fwd(x.to(gpu).contiguous(memory_format=torch.channels_last), w.to(gpu), None, (1, 1), (1, 1),
                     (1, 1), 4, out_dtype=torch.float32)
    ref = TF.conv2d(x.double(), w.double(), None, 1, 1, 1, 4)
    assert rel_err(y, ref) < 1e-5


def test_bf16_dilated_conv_dgrad(gpu):
    """bf16 dilated conv data gradient (the tuned kernel's dgrad needs
    dilation 1; the generic one takes it)."""
    from singa_amd.ops import functional as F
    x = _rand(2, 16, 12, 12, seed=32, dtype=torch.bfloat16)
    w = (_rand(16, 16, 3, 3, seed=33) * 0.2).to(torch.bfloat16)
    dy = _rand(2, 16, 8, 8, seed=34, dtype=torch.bfloat16)
    xd = x.double().requires_grad_(True)
    ref = TF.conv2d(xd, w.double(), None, 1, 0, 2)
    (gx,) = torch.autograd.grad(ref, [xd], dy.double())
    cl = torch.channels_last
    dx, _, _ = F.conv2d_bwd(x.to(gpu).contiguous(memory_format=cl), w.to(gpu).contiguous(memory_format=cl),
                            dy.to(gpu).contiguous(memory_format=cl), (1, 1), (0, 0), (2, 2), 1, need_dx=True)
    assert rel_err(dx, gx) < 1e-2


def test_fp32_linear_layer_step(gpu):
    """fp32 Linear forward/backward through autograd: no hipBLAS, exact."""
    from singa_amd import autograd, device, tensor
    dev = device.create_rocm_gpu()
    x = _rand(64, 784, seed=40)
    W = _rand(784, 250, seed=41) * 0.05
    b = _rand(250, seed=42)
    tx = tensor.from_numpy(x.numpy()).to_device(dev)
    tW = tensor.from_numpy(W.numpy()).to_device(dev)
    tW.requires_grad = tW.stores_grad = True
    tb = tensor.from_numpy(b.numpy()).to_device(dev)
    tb.requires_grad = tb.stores_grad = True
    autograd.training = True
    try:
        y = autograd.linear(tx, tW, tb)
        loss = autograd.reduce_mean(autograd.square(y), None, 0) if hasattr(autograd, "reduce_mean") else None
        grads = dict((id(p), g) for p, g in autograd.backward(y, tensor.from_numpy(np.ones((64, 250), np.float32))
                                                              .to_device(dev)))
    finally:
        autograd.training = False
    del loss
    ref = x.double() @ W.double() + b.double()
    assert rel_err(y.data, ref) < 1e-5
    assert rel_err(grads[id(tW)].data, x.double().t() @ torch.ones(64, 250, dtype=torch.float64)) < 1e-5
