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


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("splits", [0, -1, 3])
def test_fp32_gemm_every_tile_and_split(gpu, tile, splits):
    """Every fp32 tile variant and split-K mode (forced through ggemm_tune),
    with a biased plain output (split-K: zeroed C, split 0 adds the bias), an
    accumulating weight-gradient with the fused bias-gradient column sums,
    and a dgrad-shaped call -- exact to 1e-5."""
    from singa_amd.ops import functional as F
    from singa_amd.ops import native as N
    L = N.lib()
    x, w, b = _rand(300, 203, seed=11), _rand(203, 157, seed=12), _rand(157, seed=13)
    dy, acc, db0 = _rand(300, 157, seed=14), _rand(203, 157, seed=15), _rand(157, seed=16)
    try:
        L.ggemm_tune(0, tile)
        L.ggemm_tune(1, splits)
        y = F.matmul(x.to(gpu), w.to(gpu), bias=b.to(gpu))
        assert rel_err(y, x.double() @ w.double() + b.double()) < 1e-5
        g, db = acc.to(gpu), db0.to(gpu)
        F.gemm_tn_acc(x.to(gpu), dy.to(gpu), g, colsum_b=db)
        assert rel_err(g, acc.double() + x.double().t() @ dy.double()) < 1e-5
        assert rel_err(db, db0.double() + dy.double().sum(0)) < 1e-5
        dx = F.gemm_nt(dy.to(gpu), w.to(gpu))
        assert rel_err(dx, dy.double() @ w.double().t()) < 1e-5
    finally:
        L.ggemm_tune(0, 0)
        L.ggemm_tune(1, 0)


@pytest.mark.parametrize("tile", [0, 1, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("splits", [0, -1, 3])
def test_fp32_dma_gemm_every_tile_and_split(gpu, tile, splits):
    """The LDS-DMA fp32 kernel (f32d_k: 16-byte-unit operands, ragged tile
    edges, K not a multiple of the K-tile) on the three MLP GEMM layouts --
    K-major x K-outer forward with bias, K-outer x K-outer weight gradient
    with the fused bias-gradient column sums, K-major x K-major data gradient
    -- exact to 1e-5 against fp64, and the DMA kernel really ran (32-row tiles
    fall back to ggemm_k where a K-outer operand has 32 rows)."""
    from singa_amd.ops import functional as F
    from singa_amd.ops import native as N
    L = N.lib()
    x, w, b = _rand(300, 204, seed=21), _rand(204, 156, seed=22), _rand(156, seed=23)
    dy, acc, db0 = _rand(300, 156, seed=24), _rand(204, 156, seed=25), _rand(156, seed=26)
    kout_ok = tile not in (6, 7, 8)  # a K-outer operand needs >= 64 tile rows
    try:
        L.ggemm_tune(0, tile)
        L.ggemm_tune(1, splits)
        y = F.matmul(x.to(gpu), w.to(gpu), bias=b.to(gpu))
        assert rel_err(y, x.double() @ w.double() + b.double()) < 1e-5
        assert tile == 0 or L.ggemm_last_dma() == (1 if kout_ok or tile == 7 else 0)
        g, db = acc.to(gpu), db0.to(gpu)
        F.gemm_tn_acc(x.to(gpu), dy.to(gpu), g, colsum_b=db)
        assert rel_err(g, acc.double() + x.double().t() @ dy.double()) < 1e-5
        assert rel_err(db, db0.double() + dy.double().sum(0)) < 1e-5
        assert tile == 0 or L.ggemm_last_dma() == (1 if kout_ok else 0)
        dx = F.gemm_nt(dy.to(gpu), w.to(gpu))
        assert rel_err(dx, dy.double() @ w.double().t()) < 1e-5
        assert tile == 0 or L.ggemm_last_dma() == 1
    finally:
        L.ggemm_tune(0, 0)
        L.ggemm_tune(1, 0)


_ACTS = {"relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh,
         "stanh": lambda h: 1.7159047 * torch.tanh(0.66666667 * h)}


@pytest.mark.parametrize("act", sorted(_ACTS))
def test_fp32_gemm_fused_activation(gpu, act):
    """Output activation in the epilogue, and a data-gradient GEMM that also
    multiplies by the producer activation's derivative (from its output)."""
    from singa_amd.ops import functional as F
    x, w, b = _rand(150, 77, seed=51), _rand(77, 93, seed=52) * 0.2, _rand(93, seed=53)
    y = F.matmul(x.to(gpu), w.to(gpu), bias=b.to(gpu), act=act)
    ref = _ACTS[act](x.double() @ w.double() + b.double())
    assert rel_err(y, ref) < 1e-5
    dy, w2 = _rand(150, 41, seed=54), _rand(93, 41, seed=55)
    dx = F.gemm_nt(dy.to(gpu), w2.to(gpu), act_grad=(act, y))
    h = (x.double() @ w.double() + b.double()).requires_grad_(True)
    (gh,) = torch.autograd.grad(_ACTS[act](h), [h], dy.double() @ w2.double().t())
    assert rel_err(dx, gh) < 1e-5


@pytest.mark.parametrize("act", ["relu", "stanh", "sigmoid"])
def test_fp32_mlp_step_bias_grad_fused(gpu, act):
    """One SGD step (lr 1, no momentum) of an fp32 MLP whose Linear layers
    fuse the activation (forward epilogue; backward in the next layer's
    data-gradient epilogue) and take the bias gradient from the
    weight-gradient GEMM (the optimizer's flat gradient views): every
    parameter update equals the float64 PyTorch gradient of the same
    network."""
    from singa_amd import device, opt, tensor
    from singa_amd.models import mlp
    dev = device.create_rocm_gpu()
    dev.SetRandSeed(3)
    m = mlp.create_model((48, 40), 10, activation=act)
    x = _rand(130, 33, seed=31)
    y = torch.randint(0, 10, (130,), generator=torch.Generator().manual_seed(32)).int()
    tx = tensor.from_numpy(x.numpy()).to_device(dev)
    ty = tensor.from_numpy(y.numpy()).to_device(dev)
    m.set_optimizer(opt.SGD(lr=1.0))
    m.compile([tx], is_train=True, use_graph=False)
    m.train()
    before = {k: v.data.double().cpu().clone() for k, v in m.get_params().items()}
    m(tx, ty)
    torch.cuda.synchronize()
    after = {k: v.data.double().cpu() for k, v in m.get_params().items()}
    ref = {k: v.clone().requires_grad_(True) for k, v in before.items()}
    names = sorted(ref)
    ws = [n for n in names if ref[n].dim() == 2]
    bs = [n for n in names if ref[n].dim() == 1]
    assert len(ws) == 3 and len(bs) == 3
    # layer order follows the creation order of the parameters (input width 33 first)
    order = sorted(zip(ws, bs), key=lambda wb: [33, 48, 40].index(ref[wb[0]].shape[0]))
    h = x.double()
    for i, (wn, bn) in enumerate(order):
        h = h @ ref[wn] + ref[bn]
        if i < 2:
            h = _ACTS[act](h)
    loss = torch.nn.functional.cross_entropy(h, y.long())
    loss.backward()
    for n in names:
        assert rel_err(before[n] - after[n], ref[n].grad) < 1e-5, n


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


def test_lazy_grad_zero_matches_full_zero(gpu):
    """The optimizer leaves the weight-gradient slices of fp32 Linear layers
    unzeroed (their GEMMs overwrite them on the first write of a step):
    three SGD-momentum steps equal the fully-zeroed run, including a step in
    which one layer does not run (its stale slice is cleared before the
    update, so only momentum moves it)."""
    from singa_amd import autograd, device, layer, model, opt, tensor

    class Net(model.Model):
        def __init__(self):
            super().__init__()
            self.a = layer.Linear(32, activation="relu")
            self.b = layer.Linear(32, activation="relu")
            self.out = layer.Linear(10)
            self.loss_fn = layer.SoftMaxCrossEntropy()
            self.skip_b = False

        def forward(self, x):
            h = self.a(x)
            if not self.skip_b:
                h = self.b(h)
            return self.out(h)

        def train_one_batch(self, x, y):
            o = self.forward(x)
            loss = self.loss_fn(o, y)
            self.optimizer(loss)
            return o, loss

    def run(lazy):
        opt.LAZY_ZERO = lazy
        autograd.OVERWRITE_FIRST.clear()
        dev = device.create_rocm_gpu()
        dev.SetRandSeed(7)
        m = Net()
        x = tensor.from_numpy(_rand(64, 32, seed=61).numpy()).to_device(dev)
        y = tensor.from_numpy(torch.randint(0, 10, (64,), generator=torch.Generator().manual_seed(62))
                              .int().numpy()).to_device(dev)
        m.set_optimizer(opt.SGD(lr=0.1, momentum=0.9))
        m.compile([x], is_train=True, use_graph=False)
        m.train()
        for step in range(4):
            m.skip_b = step == 2
            m(x, y)
        torch.cuda.synchronize()
        return {k: v.data.double().cpu().clone() for k, v in m.get_params().items()}, len(autograd.OVERWRITE_FIRST)

    try:
        full, _ = run(False)
        lazy, n_ow = run(True)
    finally:
        opt.LAZY_ZERO = True
    assert n_ow >= 2  # the lazy path was taken
    for k in full:
        assert rel_err(lazy[k], full[k]) < 1e-6, k


@pytest.mark.parametrize("act", ["gelu", "gelu_tanh", "stanh"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_fused_activation_tuned_and_generic(gpu, act, dt):
    """bf16 (tuned kernel's LDS-staged epilogue) and fp32 GEMMs with a fused
    activation (+ the pre-activation written to act_aux) and a data-gradient
    GEMM taking the activation's derivative: equal to the separate
    elementwise kernels on the same rounded values."""
    from singa_amd.ops import functional as F
    x = _rand(256, 192, seed=71).to(gpu).to(dt)
    w = (_rand(192, 384, seed=72) * 0.1).to(gpu).to(dt)
    b = _rand(384, seed=73).to(gpu)
    z = torch.empty(256, 384, device=gpu, dtype=dt)
    y = F.matmul(x, w, out_dtype=dt, bias=b, act=act, act_aux=z)
    z_ref = F.matmul(x, w, out_dtype=dt, bias=b)
    assert rel_err(z, z_ref) < (1e-6 if dt == torch.float32 else 1e-3)
    y_ref = F.unary(act, z_ref)
    assert rel_err(y, y_ref) < (1e-6 if dt == torch.float32 else 1e-2)
    dy, w2 = _rand(256, 128, seed=74).to(gpu).to(dt), (_rand(384, 128, seed=75) * 0.1).to(gpu).to(dt)
    t = z if act in F.ACT_XFORM else y
    dz = F.gemm_nt(dy, w2, out_dtype=dt, act_grad=(act, t))
    dx = F.gemm_nt(dy, w2, out_dtype=dt)
    dz_ref = F.unary_bwd(act, z, None, dx) if act in F.ACT_XFORM else F.unary_bwd(act, None, y, dx)
    assert rel_err(dz, dz_ref) < (1e-6 if dt == torch.float32 else 1e-2)


def test_bert_layer_fused_gelu_matches_unfused(gpu):
    """A BERT encoder layer with GELU fused into fc1 / fc2's GEMM epilogues
    gives the unfused layer's output and weight gradients (bf16 tolerance)."""
    from singa_amd import autograd, device, tensor
    from singa_amd.models import bert
    dev = device.create_rocm_gpu()
    outs = []
    for fuse in (False, True):
        dev.SetRandSeed(11)
        lay = bert.EncoderLayer(64, 4, 256, dropout=0.0, fuse_gelu=fuse)
        x = tensor.from_numpy(_rand(2, 16, 64, seed=81).numpy()).to_device(dev)
        x = tensor.Tensor(data=x.data.bfloat16(), device=dev, requires_grad=False)
        autograd.training = True
        try:
            y = lay(x)
            dy = tensor.Tensor(data=_rand(*y.shape, seed=82).to(gpu).to(y.data.dtype), device=dev,
                               requires_grad=False)
            grads = {id(p): g.data.float().cpu() for p, g in autograd.backward(y, dy)}
        finally:
            autograd.training = False
        ps = lay.get_params()
        outs.append((y.data.float().cpu(), {k: grads[id(v)] for k, v in ps.items() if id(v) in grads}))
    (y0, g0), (y1, g1) = outs
    assert rel_err(y1, y0) < 2e-2
    assert set(g0) == set(g1) and len(g0) > 6
    for k in g0:
        assert rel_err(g1[k], g0[k]) < 3e-2, k


@pytest.mark.parametrize("M,N,K", [(4096, 3072, 768), (1000, 136, 64), (300, 124, 96), (777, 2048, 2304)])
def test_act_grad_gemm_output_column_sums(gpu, M, N, K):
    """A data-gradient GEMM taking its producer's activation backward also
    sums its output's columns into the producer's bias gradient (colsum_c,
    accumulated): the tuned kernel's staged epilogue where N % 8 == 0, else
    a separate pass -- equal to fp32 column sums of the bf16 output, and the
    output bitwise the call without it."""
    from singa_amd.ops import functional as F
    dy = _rand(M, K, seed=91).to(gpu).bfloat16()
    w = (_rand(N, K, seed=92) * 0.1).to(gpu).bfloat16()
    z = _rand(M, N, seed=93).to(gpu).bfloat16()
    ref = F.gemm_nt(dy, w, out_dtype=torch.bfloat16, act_grad=("gelu", z))
    cs0 = _rand(N, seed=94).to(gpu)
    cs = cs0.clone()
    out = F.gemm_nt(dy, w, out_dtype=torch.bfloat16, act_grad=("gelu", z), colsum_c=cs)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    torch.testing.assert_close(cs, cs0 + out.float().sum(0), rtol=1e-4, atol=1e-2)
