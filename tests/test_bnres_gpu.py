"""The fused residual tail relu(BN(conv1x1(y, W)) + res) with its algebraic
backward (autograd.ConvBNAddReLU, F.bnres_bwd, csrc/kernels/bnres.hip):

* one tail against a PyTorch fp32 reference of the same op (forward and
  every gradient: y, W, gamma, beta, res);
* two-source GEMM building blocks (bnres_wgrad: [g | y]^T y; bnres_dgrad:
  [g | y] B^T + bias) against fp32 matmuls;
* a chain of bottlenecks (downsample + two identity blocks) with the fused
  tail on vs. off (the unfused conv -> BN path): every parameter gradient
  agrees, and the upstream dgrad epilogue really produced the masked,
  summed gradient (no fallback mask pass for the inner block).
"""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def test_bnres_gemm_blocks(gpu):
    from singa_amd.ops import native as N

    L = N.lib()
    g0 = torch.Generator(device=gpu).manual_seed(1)
    P, K4, C = 4096, 256, 64
    g = torch.randn(P, K4, device=gpu, generator=g0).bfloat16()
    y = torch.randn(P, C, device=gpu, generator=g0).bfloat16()
    out = torch.zeros((K4 + C) * C, device=gpu)
    L.bnres_wgrad(g.data_ptr(), y.data_ptr(), out.data_ptr(), P, K4, C, N.stream())
    ref = torch.cat([g.float(), y.float()], 1).t() @ y.float()
    assert rel_err(out.view(K4 + C, C), ref) < 1e-5
    bd = (torch.randn(C, K4 + C, device=gpu, generator=g0) * 0.05).bfloat16()
    bias = torch.randn(C, device=gpu, generator=g0)
    dx = torch.empty(P, C, device=gpu, dtype=torch.bfloat16)
    L.bnres_dgrad(g.data_ptr(), y.data_ptr(), bd.data_ptr(), bias.data_ptr(), dx.data_ptr(), P, K4, C, 0, 0,
                  N.stream())
    ref = torch.cat([g.float(), y.float()], 1) @ bd.float().t() + bias
    assert rel_err(dx, ref) < 1e-2


@pytest.mark.parametrize("P,K4,C", [(6000, 512, 128), (3000, 1024, 256), (2500, 0, 128), (1800, 256, 384)])
@pytest.mark.parametrize("wide", [1, 0])
def test_bnres_wgrad_tiles(gpu, P, K4, C, wide):
    """[g | y]^T y on the 256 x 128 three-stage tiles (wide = 1: K4 % 256 == 0,
    C >= 128; K4 = 0 is the forward's Gram-only call) and on the 128 x 128
    ones, exact to fp32 accumulation against the fp32 product."""
    from singa_amd.ops import native as N

    L = N.lib()
    g0 = torch.Generator(device=gpu).manual_seed(7)
    g = torch.randn(P, max(K4, 1), device=gpu, generator=g0).bfloat16()[:, :K4].contiguous()
    y = torch.randn(P, C, device=gpu, generator=g0).bfloat16()
    out = torch.zeros((K4 + C) * C, device=gpu)
    L.bnres_tune(0, wide)
    try:
        L.bnres_wgrad(g.data_ptr() if K4 else y.data_ptr(), y.data_ptr(), out.data_ptr(), P, K4, C, N.stream())
        torch.cuda.synchronize()
    finally:
        L.bnres_tune(0, 1)
    ref = torch.cat([g.float(), y.float()], 1).t() @ y.float()
    assert rel_err(out.view(K4 + C, C), ref) < 1e-5


def test_bnres_tail_matches_fp32(gpu):
    from singa_amd import autograd as AG
    from singa_amd import device
    from singa_amd.tensor import Tensor

    dev = device.create_rocm_gpu()
    g0 = torch.Generator(device=gpu).manual_seed(7)
    Nn, C, K4, H = 8, 64, 256, 14
    y = _cl(torch.relu(torch.randn(Nn, C, H, H, device=gpu, generator=g0))).bfloat16()
    W = (torch.randn(K4, C, 1, 1, device=gpu, generator=g0) * 0.08).bfloat16().float()
    gamma = 1.0 + 0.2 * torch.randn(K4, device=gpu, generator=g0)
    beta = 0.2 * torch.randn(K4, device=gpu, generator=g0)
    res = _cl(torch.randn(Nn, K4, H, H, device=gpu, generator=g0)).bfloat16()
    dout = _cl(torch.randn(Nn, K4, H, H, device=gpu, generator=g0)).bfloat16()
    rm, rv = torch.zeros(K4, device=gpu), torch.ones(K4, device=gpu)

    AG.training = True
    try:
        ty = Tensor(data=y.clone(), device=dev, requires_grad=True, stores_grad=True)
        tW = Tensor(data=W.clone(), device=dev, requires_grad=True, stores_grad=True)
        tg = Tensor(data=gamma.clone(), device=dev, requires_grad=True, stores_grad=True)
        tb = Tensor(data=beta.clone(), device=dev, requires_grad=True, stores_grad=True)
        tr = Tensor(data=res.clone(), device=dev, requires_grad=True, stores_grad=True)
        out = AG.ConvBNAddReLU(rm, rv, 0.1, 1e-5)(ty, tW, tg, tb, tr)
        loss = AG.reduce_sum(AG.mul(out, Tensor(data=dout, device=dev, requires_grad=False)), None)
        grads = {id(p): gg.data.float().clone() for p, gg in AG.backward(loss)}
    finally:
        AG.training = False

    yr = y.float().requires_grad_(True)
    Wr = W.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    rr = res.float().requires_grad_(True)
    c = TF.conv2d(yr, Wr)
    mean = c.mean((0, 2, 3), keepdim=True)
    var = c.var((0, 2, 3), unbiased=False, keepdim=True)
    pre = gr.view(1, -1, 1, 1) * (c - mean) / torch.sqrt(var + 1e-5) + br.view(1, -1, 1, 1) + rr
    assert rel_err(out.data, torch.relu(pre).detach()) < 1e-2
    # the ReLU mask of OUR (bf16) forward: elements within bf16 rounding of 0
    # may flip against an fp32 forward, which alone moves every gradient by a
    # few percent -- the backward is checked on the same mask
    o = pre * (out.data > 0).float()
    (o * dout.float()).sum().backward()
    errs = {"y": rel_err(grads[id(ty)], yr.grad), "W": rel_err(grads[id(tW)], Wr.grad),
            "gamma": rel_err(grads[id(tg)], gr.grad), "beta": rel_err(grads[id(tb)], br.grad),
            "res": rel_err(grads[id(tr)], rr.grad)}
    print(errs)
    assert max(errs.values()) < 2e-2, errs


@pytest.mark.parametrize("stride", [1, 2])
def test_bnres_chain_matches_unfused(gpu, stride):
    """downsample block (ConvBNDualAddReLU: both tail branches algebraic, a
    strided shortcut through strided_pick / strided_place) + two identity
    blocks (ConvBNAddReLU), fused vs. the unfused conv -> BN path"""
    from singa_amd import autograd as AG
    from singa_amd import device
    from singa_amd.models.resnet import Bottleneck
    from singa_amd.ops import functional as FF
    from singa_amd.tensor import Tensor

    dev = device.create_rocm_gpu()
    dev.SetRandSeed(11)
    blks = [Bottleneck(64, stride, True), Bottleneck(64, 1, False), Bottleneck(64, 1, False)]
    g0 = torch.Generator(device=gpu).manual_seed(4)
    xf = torch.randn(8, 128, 14 * stride, 14 * stride, device=gpu, generator=g0)
    dyt = None
    on0 = FF.BNRES
    calls = {"bwd": 0, "masksum": 0}
    orig_bwd, orig_ms = FF.bnres_bwd, FF.bnres_masksum

    def spy_bwd(*a, **k):
        calls["bwd"] += 1
        return orig_bwd(*a, **k)

    def spy_ms(*a, **k):
        calls["masksum"] += 1
        return orig_ms(*a, **k)

    def run(on):
        nonlocal dyt
        FF.BNRES = on
        AG.training = True
        x = Tensor(data=_cl(xf).bfloat16(), device=dev, requires_grad=True, stores_grad=False)
        try:
            h = x
            for b in blks:
                h = b(h)
            if dyt is None:
                dyt = torch.randn(h.shape, device=gpu, generator=g0)
            loss_t = AG.reduce_sum(AG.mul(h, Tensor(data=_cl(dyt).bfloat16(), device=dev, requires_grad=False)),
                                   None)
            gr = {id(p): gg.data.float().clone() for p, gg in AG.backward(loss_t)}
        finally:
            AG.training = False
            FF.BNRES = on0
        return gr

    run(False)  # creates the parameters
    FF.bnres_bwd, FF.bnres_masksum = spy_bwd, spy_ms
    try:
        g_on = run(True)
    finally:
        FF.bnres_bwd, FF.bnres_masksum = orig_bwd, orig_ms
    g_off = run(False)
    # the two identity blocks ran fused, the downsample block's two branches
    # too; only the last block (fed by the loss, no consuming conv) needed the
    # fallback mask pass
    assert calls == {"bwd": 4, "masksum": 1}, calls
    # both paths against fp32 PyTorch: a few ReLU bits flip between any two
    # bf16 runs (atomic-order rounding) and, under a random output gradient,
    # move every gradient of this small chain by a few percent -- so the fused
    # path must be as close to fp32 as the unfused one, not equal to it
    named = [(f"{i}.{k}", p) for i, b in enumerate(blks) for k, p in b.get_params().items()]
    leaves = {n: p.data.float().clone().requires_grad_(True) for n, p in named}
    saved = {n: p.data for n, p in named}
    for n, p in named:
        p.data = leaves[n]
    try:
        h = _cl(xf).bfloat16().float()
        for b in blks:
            h = _torch_bottleneck(b, h)
        (h * _cl(dyt).bfloat16().float()).sum().backward()
    finally:
        for n, p in named:
            p.data = saved[n]
    e_on = {n: rel_err(g_on[id(p)], leaves[n].grad) for n, p in named}
    e_off = {n: rel_err(g_off[id(p)], leaves[n].grad) for n, p in named}
    print({n: (round(e_on[n], 4), round(e_off[n], 4)) for n in e_on})
    for n in e_on:
        assert e_on[n] <= 1.5 * e_off[n] + 2e-2, (n, e_on[n], e_off[n])


@pytest.mark.parametrize("C,K4", [(64, 256), (128, 512)])
def test_bnres_recompute_forward_matches_unfused(gpu, C, K4):
    """The recomputed tail forward (F.bnres_fwd: statistics-only GEMM pass,
    then BN + residual + ReLU + mask in the second pass's epilogue) against
    the unfused conv -> BN apply: same output, mask, running statistics and
    gradients (up to the atomic-order rounding of the statistics)."""
    from singa_amd import autograd as AG
    from singa_amd import device
    from singa_amd.ops import functional as FF
    from singa_amd.ops import native as N
    from singa_amd.tensor import Tensor

    dev = device.create_rocm_gpu()
    g0 = torch.Generator(device=gpu).manual_seed(3)
    Nn, H = (42, 56) if C == 64 else (168, 28)  # enough 128-row tiles for the persistent kernel
    y = _cl(torch.relu(torch.randn(Nn, C, H, H, device=gpu, generator=g0))).bfloat16()
    W = (torch.randn(K4, C, 1, 1, device=gpu, generator=g0) * 0.08).bfloat16()
    gamma = 1.0 + 0.2 * torch.randn(K4, device=gpu, generator=g0)
    beta = 0.2 * torch.randn(K4, device=gpu, generator=g0)
    res = _cl(torch.randn(Nn, K4, H, H, device=gpu, generator=g0)).bfloat16()
    dout = _cl(torch.randn(Nn, K4, H, H, device=gpu, generator=g0)).bfloat16()
    assert N.lib().sk_tail_ok(Nn * H * H, K4, C)
    calls = [0]
    orig = FF.bnres_fwd

    def spy(*a, **k):
        r = orig(*a, **k)
        calls[0] += r is not None
        return r

    def run(on):
        FF.TAIL_RECOMPUTE = on
        rm, rv = torch.zeros(K4, device=gpu), torch.ones(K4, device=gpu)
        AG.training = True
        try:
            ts = [Tensor(data=t.clone(), device=dev, requires_grad=True, stores_grad=True)
                  for t in (y, W.float(), gamma, beta, res)]
            op = AG.ConvBNAddReLU(rm, rv, 0.1, 1e-5)
            out = op(*ts)
            mask = op.st.mask.clone()
            loss = AG.reduce_sum(AG.mul(out, Tensor(data=dout, device=dev, requires_grad=False)), None)
            gr = {id(p): gg.data.float().clone() for p, gg in AG.backward(loss)}
        finally:
            AG.training = False
        return out.data.float(), mask, rm, rv, [gr[id(t)] for t in ts]

    on0 = FF.TAIL_RECOMPUTE
    FF.bnres_fwd = spy
    try:
        o1, m1, rm1, rv1, g1 = run(True)
        assert calls[0] == 1
        o0, m0, rm0, rv0, g0_ = run(False)
        assert calls[0] == 1  # (the unfused run did not take it)
    finally:
        FF.bnres_fwd = orig
        FF.TAIL_RECOMPUTE = on0
    assert rel_err(o1, o0) < 2e-3
    assert (m1 != m0).float().mean().item() < 1e-3
    assert rel_err(rm1, rm0) < 1e-4 and rel_err(rv1, rv0) < 1e-4
    errs = [rel_err(a, b) for a, b in zip(g1, g0_)]
    print(errs)
    assert max(errs) < 1e-2, errs


def test_strided_pick_place(gpu):
    from singa_amd.ops import functional as FF

    g0 = torch.Generator(device=gpu).manual_seed(5)
    for (n, c, h, w, st) in ((2, 64, 7, 9, 2), (3, 256, 56, 56, 2), (1, 128, 5, 5, 3)):
        x = _cl(torch.randn(n, c, h, w, device=gpu, generator=g0)).bfloat16()
        xs = FF.strided_pick(x, st)
        assert torch.equal(xs, x[:, :, ::st, ::st])
        full = FF.strided_place(xs, x.shape, st)
        ref = torch.zeros_like(x)
        ref[:, :, ::st, ::st] = xs
        assert torch.equal(full, ref)


def test_strided_shortcut_grad_absorbed_by_conv1(gpu):
    """The compact strided shortcut gradient (F.StridedGrad): (a) a 1x1 conv's
    fused-tail dgrad (gmask path) adds it from the compact tensor exactly as it
    adds the placed full-grid tensor; (b) in a chain -- a stride-2 downsample
    block fed by a fused tail -- the engine hands it to the block's conv1 and
    nothing is ever placed on the full grid."""
    import numpy as np

    from singa_amd import autograd as AG
    from singa_amd import device
    from singa_amd.models.resnet import Bottleneck
    from singa_amd.ops import functional as FF
    from singa_amd.tensor import Tensor

    g0 = torch.Generator(device=gpu).manual_seed(6)
    Nn, C, K, H = 8, 256, 64, 28
    x = _cl(torch.randn(Nn, C, H, H, device=gpu, generator=g0)).bfloat16()
    w = (torch.randn(K, C, 1, 1, device=gpu, generator=g0) * 0.05).bfloat16()
    dy = _cl(torch.randn(Nn, K, H, H, device=gpu, generator=g0)).bfloat16()
    gc = _cl(torch.randn(Nn, C, H // 2, H // 2, device=gpu, generator=g0)).bfloat16()
    gmask = torch.randint(0, 256, (Nn * H * H * C // 8,), device=gpu, dtype=torch.uint8, generator=g0)
    outs = []
    for lazy in (True, False):
        acc = FF.StridedGrad(gc, 2, x.shape) if lazy else FF.strided_place(gc, tuple(x.shape), 2)
        dx, _, _ = FF.conv2d_bwd(x, w, dy, (1, 1), (0, 0), (1, 1), 1, need_dx=True, dx_acc=acc,
                                 bn_producer=("gmask", gmask))
        assert getattr(dx, "_sg_absorbed", None) is acc
        outs.append((dx.float(), dx._sg_gsum[0].clone()))
    assert torch.equal(outs[0][0], outs[1][0])  # the same bf16 values, added from the compact tensor
    assert rel_err(outs[0][1], outs[1][1]) < 1e-5  # (the masked sums: atomic order only)

    dev = device.create_rocm_gpu()
    dev.SetRandSeed(13)
    blks = [Bottleneck(64, 1, True), Bottleneck(64, 2, True), Bottleneck(64, 1, False)]
    xf = torch.randn(8, 128, 28, 28, device=gpu, generator=g0)
    places = [0]
    orig_place = FF.strided_place

    def spy_place(*a, **k):
        places[0] += 1
        return orig_place(*a, **k)

    AG.training = True
    try:
        xt = Tensor(data=_cl(xf).bfloat16(), device=dev, requires_grad=True, stores_grad=False)
        h = xt
        for b in blks:
            h = b(h)
        dyt = torch.randn(h.shape, device=gpu, generator=g0)
        FF.strided_place = spy_place
        loss_t = AG.reduce_sum(AG.mul(h, Tensor(data=_cl(dyt).bfloat16(), device=dev, requires_grad=False)), None)
        gr = [gg.data.float() for _, gg in AG.backward(loss_t)]
    finally:
        FF.strided_place = orig_place
        AG.training = False
    assert places[0] == 0, places
    assert len(gr) > 30 and all(np.isfinite(float(t.norm())) for t in gr)


def _torch_bottleneck(blk, x):
    """fp32 PyTorch reference of a Bottleneck (training-mode BN, batch statistics)."""
    def bn(t, layer, relu):
        y = TF.batch_norm(t, None, None, layer.scale.data.float(), layer.bias.data.float(), True, 0.0, layer.eps)
        return torch.relu(y) if relu else y
    o = bn(TF.conv2d(x, blk.conv1.W.data.float()), blk.bn1, True)
    o = bn(TF.conv2d(o, blk.conv2.W.data.float(), stride=blk.conv2.stride, padding=1), blk.bn2, True)
    o = bn(TF.conv2d(o, blk.conv3.W.data.float()), blk.bn3, False)
    sc = (bn(TF.conv2d(x, blk.down_conv.W.data.float(), stride=blk.down_conv.stride), blk.down_bn, False)
          if blk.has_down else x)
    return torch.relu(o + sc)


def test_dual_tail_recompute_matches_unfused(gpu):
    """ResNet-50's stage-1 downsample block (stride 1, 64 -> 256): the
    recomputed two-branch tail forward (F.bnres_dual_fwd: statistics passes,
    then one two-source GEMM with the BN scales folded into the weights) vs.
    the stored-output forward.  The folded weights round differently (not
    bitwise), so a few outputs near 0 flip their ReLU mask and, under a random
    output gradient, every parameter gradient moves by a few percent; the
    check is therefore that both paths are equally close to fp32 PyTorch."""
    from singa_amd import autograd as AG
    from singa_amd import device
    from singa_amd.models.resnet import Bottleneck
    from singa_amd.ops import functional as FF
    from singa_amd.tensor import Tensor

    dev = device.create_rocm_gpu()
    dev.SetRandSeed(17)
    blk = Bottleneck(64, 1, True)
    g0 = torch.Generator(device=gpu).manual_seed(8)
    xf = torch.relu(torch.randn(42, 64, 56, 56, device=gpu, generator=g0))  # 131712 pixels: the persistent kernel
    dyt = torch.randn(42, 256, 56, 56, device=gpu, generator=g0)
    calls = [0]
    orig = FF.bnres_dual_fwd

    def spy(*a, **k):
        r = orig(*a, **k)
        calls[0] += r is not None
        return r

    def run(on):
        r0 = FF.TAIL_RECOMPUTE
        FF.TAIL_RECOMPUTE = on
        AG.training = True
        try:
            x = Tensor(data=_cl(xf).bfloat16(), device=dev, requires_grad=True, stores_grad=False)
            h = blk(x)
            out = h.data.float().clone()
            loss_t = AG.reduce_sum(AG.mul(h, Tensor(data=_cl(dyt).bfloat16(), device=dev, requires_grad=False)),
                                   None)
            gr = {id(p): gg.data.float().clone() for p, gg in AG.backward(loss_t)}
        finally:
            AG.training = False
            FF.TAIL_RECOMPUTE = r0
        return out, gr

    run(False)
    FF.bnres_dual_fwd = spy
    try:
        o1, g1 = run(True)
    finally:
        FF.bnres_dual_fwd = orig
    assert calls[0] == 1
    o0, g0_ = run(False)
    assert rel_err(o1, o0) < 1e-2
    assert float(((o1 > 0) != (o0 > 0)).float().mean()) < 2e-3
    params = blk.get_params()
    leaves = {k: p.data.float().clone().requires_grad_(True) for k, p in params.items()}
    saved = {k: p.data for k, p in params.items()}
    for k, p in params.items():
        p.data = leaves[k]
    try:
        ref = _torch_bottleneck(blk, xf.bfloat16().float())
        (ref * dyt.bfloat16().float()).sum().backward()
    finally:
        for k, p in params.items():
            p.data = saved[k]
    assert rel_err(o1, ref.detach()) < 1e-2 and rel_err(o0, ref.detach()) < 1e-2
    e_on = {k: rel_err(g1[id(p)], leaves[k].grad) for k, p in params.items()}
    e_off = {k: rel_err(g0_[id(p)], leaves[k].grad) for k, p in params.items()}
    print({k: (round(e_on[k], 4), round(e_off[k], 4)) for k in e_on})
    for k in e_on:
        assert e_on[k] <= 1.5 * e_off[k] + 1e-2, (k, e_on[k], e_off[k])


@pytest.mark.parametrize("K,C,H,Nn", [(64, 256, 56, 42), (128, 512, 28, 168)])
def test_gsum_dgrad_persistent_matches_fp32(gpu, K, C, H, Nn):
    """The fused-tail output gradient of a 1x1 conv on the persistent kernel
    (sk_gemm_k EPI 2: (dgrad + acc) * mask bit, column sums) against fp32 and
    against the generic kernel's epilogue (knob 9 off)."""
    from singa_amd.ops import functional as FF
    from singa_amd.ops import native as N

    g0 = torch.Generator(device=gpu).manual_seed(21)
    x = _cl(torch.randn(Nn, C, H, H, device=gpu, generator=g0)).bfloat16()
    w = (torch.randn(K, C, 1, 1, device=gpu, generator=g0) * 0.1).bfloat16()
    dy = _cl(torch.randn(Nn, K, H, H, device=gpu, generator=g0)).bfloat16()
    acc = _cl(torch.randn(Nn, C, H, H, device=gpu, generator=g0)).bfloat16()
    gmask = torch.randint(0, 256, (Nn * H * H * C // 8,), device=gpu, dtype=torch.uint8, generator=g0)
    bits = ((gmask.view(-1, 1).int() >> torch.arange(8, device=gpu).view(1, 8)) & 1).view(Nn, H, H, C)
    ref = (TF.conv_transpose2d(dy.float(), w.float()) + acc.float()) * bits.permute(0, 3, 1, 2).float()
    res = {}
    for sk in (1, 0):
        N.lib().set_tuning(9, sk)
        try:
            dx, _, _ = FF.conv2d_bwd(x, w, dy, (1, 1), (0, 0), (1, 1), 1, need_dx=True, dx_acc=acc.clone(),
                                     bn_producer=("gmask", gmask))
        finally:
            N.lib().set_tuning(9, 1)
        gs = dx._sg_gsum[0].view(32, 2, C)[:, 0].sum(0)
        res[sk] = (dx.float(), gs)
        assert rel_err(dx, ref) < 1e-2, (sk, rel_err(dx, ref))
        assert rel_err(gs, ref.sum((0, 2, 3))) < 1e-2
    assert rel_err(res[1][0], res[0][0]) < 1e-2


@pytest.mark.parametrize("shift", [0.0, 4.0])
def test_tail_gram_statistics_large_mean(gpu, shift):
    """The residual tail's BN statistics from Gram(y) / colsum(y) (the default,
    ops/functional.py tail_stats_ws) against the statistics-only GEMM pass and
    an fp32 reference, for post-ReLU inputs whose channel means dwarf their
    spread (var = W^T Gram W / P - mean^2 cancels): the variance stays within
    the statistics pass's own distance from fp32 (plus a small absolute slack)."""
    from singa_amd.ops import functional as FF
    from singa_amd.ops import native as N

    C, K4, Nn, H = 64, 256, 42, 56
    g0 = torch.Generator(device=gpu).manual_seed(11)
    y = _cl(torch.relu(shift + 0.3 * torch.randn(Nn, C, H, H, device=gpu, generator=g0))).bfloat16()
    W = _cl((torch.randn(K4, C, 1, 1, device=gpu, generator=g0) * 0.08)).bfloat16()
    M = Nn * H * H
    L = N.lib()
    assert L.sk_tail_ok(M, K4, C)
    c = y.float().permute(0, 2, 3, 1).reshape(M, C) @ W.float().reshape(K4, C).t()
    var_ref = c.var(0, unbiased=False)
    out = {}
    old = FF.GRAM_STATS
    try:
        for gram in (True, False):
            FF.GRAM_STATS = gram
            ws, rows = FF.tail_stats_ws(y, W, M, C, K4)
            gamma, beta = torch.ones(K4, device=gpu), torch.zeros(K4, device=gpu)
            rm, rv = torch.zeros(K4, device=gpu), torch.ones(K4, device=gpu)
            p = torch.empty(4 * K4, device=gpu)
            L.bn_fwd_from_ws(ws.data_ptr(), rows, gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                             p[:K4].data_ptr(), p[K4:2 * K4].data_ptr(), p[2 * K4:3 * K4].data_ptr(),
                             p[3 * K4:].data_ptr(), M, K4, 0.1, 1e-5, N.stream())
            torch.cuda.synchronize()
            var = 1.0 / p[K4:2 * K4] ** 2 - 1e-5
            out[gram] = (p[:K4].clone(), var.clone())
    finally:
        FF.GRAM_STATS = old
    torch.testing.assert_close(out[True][0], c.mean(0), rtol=1e-3, atol=1e-3)
    e_gram = float(((out[True][1] - var_ref).abs() / var_ref).max())
    e_pass = float(((out[False][1] - var_ref).abs() / var_ref).max())
    print({"shift": shift, "gram": e_gram, "stats_pass": e_pass, "mean/std": float((c.mean(0).abs() / var_ref.sqrt()).max())})
    assert e_gram <= 2 * e_pass + 1e-2, (e_gram, e_pass)
