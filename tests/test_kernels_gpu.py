"""Numerics of every hand-written gfx950 kernel against a plain PyTorch fp32
reference of the same op (run on the MI355X box: ``pytest -m gpu``)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def bf(x):
    return x.to(torch.bfloat16)


# --------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 512, 384), (100, 72, 40), (1000, 2048, 512),
                                   (7, 8, 16), (333, 256, 1024)])
@pytest.mark.parametrize("ako,bko", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_orientations(gpu, M, N, K, ako, bko):
    from singa_amd.ops import native as NT
    if (ako and M % 8) or (bko and N % 8):
        pytest.skip("K-outer operands need rows % 8 == 0")
    g = torch.Generator(device="cpu").manual_seed(0)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    a = bf(A.t().contiguous() if ako else A).to(gpu)
    b = bf(B.t().contiguous() if bko else B).to(gpu)
    c = torch.empty(M, N, dtype=torch.float32, device=gpu)
    lda = M if ako else K
    ldb = N if bko else K
    NT.lib().gemm(a.data_ptr(), lda, ako, b.data_ptr(), ldb, bko, c.data_ptr(), N, M, N, K, 1.0, 0.0, 0, 0, 1, 1,
                  1, 0, 0, 0, NT.stream())
    ref = bf(A).float() @ bf(B).float().t()
    assert rel_err(c, ref) < 1e-5


def test_gemm_asymmetric_identity(gpu):
    """A = I with an asymmetric B catches transposed epilogue writes."""
    from singa_amd.ops import functional as F
    n = 128
    A = torch.eye(n)
    B = torch.arange(n * n, dtype=torch.float32).reshape(n, n) % 97 - 48
    c = F.matmul(bf(A).to(gpu), bf(B).to(gpu), out_dtype=torch.float32)
    assert torch.equal(c.cpu(), bf(B).float())


def test_gemm_bias_relu_bf16_out_batched(gpu):
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(1)
    a = torch.randn(3, 200, 64, generator=g)
    b = torch.randn(3, 64, 136, generator=g)
    out = F.matmul(bf(a).to(gpu), bf(b).to(gpu), out_dtype=torch.bfloat16)
    ref = bf(a).float() @ bf(b).float()
    assert rel_err(out, ref) < 8e-3
    a2, b2 = torch.randn(64, 96, generator=g), torch.randn(96, 256, generator=g)
    bias = torch.randn(256, generator=g)
    out2 = F.matmul(bf(a2).to(gpu), bf(b2).to(gpu), out_dtype=torch.float32, bias=bias.to(gpu), relu=True)
    ref2 = torch.relu(bf(a2).float() @ bf(b2).float() + bias)
    assert rel_err(out2, ref2) < 1e-5


def test_gemm_splitk_atomic(gpu):
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(2)
    a = torch.randn(4096, 64, generator=g)  # [K, M]
    b = torch.randn(4096, 96, generator=g)  # [K, N]
    out = torch.zeros(64, 96, device=gpu)
    F.gemm_tn_acc(bf(a).to(gpu), bf(b).to(gpu), out)
    ref = bf(a).float().t() @ bf(b).float()
    assert rel_err(out, ref) < 1e-5


# --------------------------------------------------------------- convolution
CONV_CASES = [
    # N, C, H, W, K, R, S, stride, pad
    (2, 64, 14, 14, 64, 1, 1, 1, 0),
    (2, 64, 14, 14, 128, 3, 3, 1, 1),
    (2, 64, 15, 15, 128, 3, 3, 2, 1),
    (2, 128, 14, 14, 256, 1, 1, 2, 0),
    (2, 3, 32, 32, 64, 7, 7, 2, 3),     # stem, C padded to 8
    (3, 20, 12, 12, 50, 5, 5, 1, 0),    # LeNet conv2: C and K not multiples of 8
    (2, 32, 9, 11, 40, 3, 3, 1, 2),
    # AlexNet: 11x11/4 stem (C padded to 8), 5x5 pad 2, 3x3 at 13x13
    (2, 3, 67, 67, 96, 11, 11, 4, 2),
    (4, 3, 224, 224, 96, 11, 11, 4, 2),
    (2, 96, 27, 27, 256, 5, 5, 1, 2),
    (2, 256, 13, 13, 384, 3, 3, 1, 1),
    # ResNet-sized spatial extents: wgrad's stepping pixel decomposition
    # (output rows >= 16 / 32 pixels) and the 128-row tiles
    (2, 64, 56, 56, 64, 3, 3, 1, 1),
    (2, 64, 56, 56, 256, 1, 1, 1, 0),
    (2, 256, 56, 56, 128, 1, 1, 2, 0),
    (2, 128, 56, 56, 128, 3, 3, 2, 1),
    (1, 32, 70, 70, 64, 3, 3, 1, 1),
    # fewer output pixels per image than a K-tile (64): wgrad's pixel walk
    # carries across whole images per tile
    (3, 64, 7, 7, 128, 3, 3, 1, 1),
    (4, 64, 5, 5, 64, 3, 3, 1, 1),
    (5, 32, 9, 9, 64, 3, 3, 2, 1),
]


@pytest.mark.parametrize("kmajor", [True, False])
@pytest.mark.parametrize("wmode", [0, 1, 5])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_bwd(gpu, case, wmode, kmajor, monkeypatch):
    from singa_amd.ops import functional as F
    from singa_amd.ops import native as NN
    monkeypatch.setattr(F, "DGRAD_KMAJOR", kmajor)  # dgrad B operand: transposed K-major copy / LDS transpose
    NN.lib().set_tuning(0, wmode)  # wgrad tile policy: 64-tiles + splits / largest tiles / measured default
    N_, C, H, W, K, R, S, st, pd = case
    g = torch.Generator().manual_seed(3)
    x = bf(torch.randn(N_, C, H, W, generator=g)).float()
    w = bf(torch.randn(K, C, R, S, generator=g) * (1.0 / math.sqrt(C * R * S))).float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = TF.conv2d(xr, wr, None, st, pd)
    dy = bf(torch.randn(yr.shape, generator=g)).float()
    yr.backward(dy)
    xg = x.to(gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wg = w.to(gpu)
    y = F.conv2d_fwd(xg, wg, None, (st, st), (pd, pd), out_dtype=torch.float32)
    assert y.shape == yr.shape
    assert rel_err(y, yr.detach()) < 1e-5
    dyg = dy.to(gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dw_acc = torch.zeros(K, C, R, S, device=gpu)
    dx, dw, db = F.conv2d_bwd(xg.float().contiguous(memory_format=torch.channels_last), wg, dyg, (st, st),
                              (pd, pd), need_dx=True, dw_out=dw_acc, need_db=True)
    NN.lib().set_tuning(0, 5)
    # bf16 outputs (the LDS-staged epilogue): fwd and dgrad
    yb = F.conv2d_fwd(xg, wg, None, (st, st), (pd, pd), out_dtype=torch.bfloat16)
    assert yb.dtype == torch.bfloat16 and rel_err(yb.float(), yr.detach()) < 1e-2
    dxb = F.conv2d_bwd(xg, wg, dyg, (st, st), (pd, pd), need_dx=True)[0]
    assert dxb.dtype == torch.bfloat16 and rel_err(dxb.float(), xr.grad) < 1e-2
    assert rel_err(dx, xr.grad) < 1e-5
    assert rel_err(dw_acc, wr.grad) < 1e-5
    assert rel_err(db, dy.sum((0, 2, 3))) < 1e-5


@pytest.mark.parametrize("case", [(2, 64, 28, 28, 256, 3, 3, 1, 1), (2, 128, 14, 14, 512, 3, 3, 1, 1),
                                  (2, 128, 28, 28, 128, 3, 3, 1, 1), (2, 512, 14, 14, 128, 1, 1, 1, 0),
                                  (2, 256, 28, 28, 256, 1, 1, 1, 0), (3, 128, 15, 15, 384, 3, 3, 2, 1)])
def test_conv_wgrad_256x128_ring(gpu, case):
    """The 8-wave weight gradient on 256 x 128 tiles (tuning knob 15: 64 x 64
    wave tiles, the compile-time three-stage ring, split-K atomics) == the
    fp32 PyTorch weight gradient of the same bf16-rounded operands."""
    from singa_amd.ops import functional as F
    from singa_amd.ops import native as NN
    N_, C, H, W, K, R, S, st, pd = case
    g = torch.Generator().manual_seed(5)
    x = bf(torch.randn(N_, C, H, W, generator=g)).float()
    w = bf(torch.randn(K, C, R, S, generator=g) * (1.0 / math.sqrt(C * R * S))).float()
    wr = w.clone().requires_grad_(True)
    yr = TF.conv2d(x, wr, None, st, pd)
    dy = bf(torch.randn(yr.shape, generator=g)).float()
    yr.backward(dy)
    xg = x.to(gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dyg = dy.to(gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for knob, k17 in ((1, 0), (0, 0), (1, 1)):  # 256 x 128 (default), 128 x 128, 128 x 256 for K_out < 256
        NN.lib().set_tuning(15, knob)
        NN.lib().set_tuning(17, k17)
        try:
            dw_acc = torch.zeros(K, C, R, S, device=gpu)
            F.conv2d_bwd(xg, w.to(gpu), dyg, (st, st), (pd, pd), need_dx=False, dw_out=dw_acc)
            torch.cuda.synchronize()
        finally:
            NN.lib().set_tuning(15, 1)
            NN.lib().set_tuning(17, 0)
        assert rel_err(dw_acc, wr.grad) < 1e-5


@pytest.fixture
def big_tiles():
    """Force an 8-wave conv/GEMM variant (5: 128x128 two workgroups per CU,
    6: 256x64 4-stage ring, 7: 256x128 3-stage ring, 8: the ping-pong 256x256
    kernel where it applies -- plain K-major GEMMs, 1x1 stride-1 conv forward
    and data gradient -- else 5) for every problem size, restore the size
    policy after."""
    from singa_amd.ops import native as NN
    yield lambda mode: NN.lib().set_tuning(4, mode)
    NN.lib().set_tuning(4, 0)


@pytest.mark.parametrize("tile", [5, 6, 7, 8])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_big_tiles(gpu, case, tile, big_tiles, monkeypatch):
    """fwd (fp32 and bf16 epilogue) and dgrad (both B-operand paths) of the
    8-wave kernels vs a PyTorch fp32 reference, including partial tiles,
    per-lane taps (C % 64 != 0) and stride phases."""
    from singa_amd.ops import functional as F
    N_, C, H, W, K, R, S, st, pd = case
    g = torch.Generator().manual_seed(5)
    x = bf(torch.randn(N_, C, H, W, generator=g)).float()
    w = bf(torch.randn(K, C, R, S, generator=g) * (1.0 / math.sqrt(C * R * S))).float()
    xr = x.clone().requires_grad_(True)
    yr = TF.conv2d(xr, w, None, st, pd)
    dy = bf(torch.randn(yr.shape, generator=g)).float()
    yr.backward(dy)
    xg = x.to(gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wg = w.to(gpu)
    dyg = dy.to(gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    big_tiles(tile)
    y = F.conv2d_fwd(xg, wg, None, (st, st), (pd, pd), out_dtype=torch.float32)
    assert rel_err(y, yr.detach()) < 1e-5
    yb = F.conv2d_fwd(xg, wg, None, (st, st), (pd, pd), out_dtype=torch.bfloat16)
    assert rel_err(yb.float(), yr.detach()) < 1e-2
    for kmajor in (True, False):
        monkeypatch.setattr(F, "DGRAD_KMAJOR", kmajor)
        dx = F.conv2d_bwd(xg.float().contiguous(memory_format=torch.channels_last), wg, dyg, (st, st), (pd, pd),
                          need_dx=True)[0]
        assert rel_err(dx, xr.grad) < 1e-5
        dxb = F.conv2d_bwd(xg, wg, dyg, (st, st), (pd, pd), need_dx=True)[0]
        assert rel_err(dxb.float(), xr.grad) < 1e-2


@pytest.mark.parametrize("tile", [5, 6, 7, 8])
@pytest.mark.parametrize("det", [False, True])
@pytest.mark.parametrize("R", [3, 1])
def test_conv_big_tiles_bn_stats(gpu, tile, det, R, big_tiles):
    import singa_amd
    from singa_amd.ops import functional as F
    singa_amd.set_deterministic(det)
    try:
        g = torch.Generator(device=gpu).manual_seed(2)
        x = torch.randn(8, 64, 28, 28, device=gpu, generator=g).bfloat16().contiguous(
            memory_format=torch.channels_last)
        w = (torch.randn(192, 64, R, R, device=gpu, generator=g) * 0.05).bfloat16().contiguous(
            memory_format=torch.channels_last)
        pd = (R // 2, R // 2)
        big_tiles(tile)
        y1 = F.conv2d_fwd(x, w, None, (1, 1), pd, out_dtype=torch.bfloat16, bn_stats=True)
        big_tiles(0)
        y2 = F.conv2d_fwd(x, w, None, (1, 1), pd, out_dtype=torch.bfloat16)
        assert rel_err(y1.float(), y2.float()) < 1e-2
        gam, bet = torch.rand(192, device=gpu) + 0.5, torch.randn(192, device=gpu)
        outs = []
        for y in (y1, y2):
            rm, rv = torch.zeros(192, device=gpu), torch.ones(192, device=gpu)
            out, st = F.batchnorm_fwd(y, gam, bet, rm, rv, True, 0.1, 1e-5, relu=True)
            outs.append((st.mean.clone(), st.invstd.clone(), rm, rv))
    finally:
        singa_amd.set_deterministic(False)
    for a, b in zip(outs[0], outs[1]):
        assert rel_err(a, b) < 1e-3


@pytest.mark.parametrize("tile", [5, 6, 7, 8])
@pytest.mark.parametrize("Nb,C,K,H,R,st", [(3, 64, 256, 14, 1, 1), (2, 128, 128, 15, 3, 2), (2, 96, 40, 9, 3, 1),
                                           (4, 256, 64, 7, 1, 2), (2, 8, 64, 33, 7, 2)])
def test_conv_big_tiles_stay_in_bounds(gpu, Nb, C, K, H, R, st, tile, big_tiles):
    from singa_amd.ops import native as NN
    L = NN.lib()
    big_tiles(tile)
    pad = R // 2
    Ho = (H + 2 * pad - R) // st + 1
    g = torch.Generator(device=gpu).manual_seed(9)
    x = torch.randn(Nb * H * H * C, device=gpu, generator=g).bfloat16()
    w = (torch.randn(K * R * R * C, device=gpu, generator=g) * 0.05).bfloat16()
    dy = torch.randn(Nb * Ho * Ho * K, device=gpu, generator=g).bfloat16()
    s = NN.stream()
    for stats in (False, True):
        y, chk = _guarded(Nb * Ho * Ho * K, torch.bfloat16, gpu)
        ws = None
        if stats:
            rows = L.conv_stats_rows(Nb * Ho * Ho, K)
            ws, wchk = _guarded(max(rows, 1) * 2 * K, torch.float32, gpu)
            ws.zero_()
        L.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, Nb, H, H, C, K, R, R, Ho, Ho, st, st, pad, pad, 1, 1,
                   0, 0, s, ws.data_ptr() if ws is not None else 0)
        chk("conv_fwd")
        if ws is not None:
            wchk("conv_fwd stats")
    if st * st <= 16:
        dx, chk = _guarded(Nb * H * H * C, torch.bfloat16, gpu)
        L.conv_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), Nb, H, H, C, K, R, R, Ho, Ho, st, st, pad, pad, 1, 1, 0,
                     s)
        chk("conv_dgrad")


@pytest.mark.parametrize("tile", [5, 6, 7, 8])
@pytest.mark.parametrize("M,N,K,ak,bk", [(300, 200, 136, 0, 0), (513, 64, 96, 0, 1), (264, 384, 64, 1, 0),
                                         (1000, 136, 200, 1, 1)])
def test_gemm_big_tiles(gpu, M, N, K, ak, bk, tile, big_tiles):
    from singa_amd.ops import native as NN
    g = torch.Generator(device=gpu).manual_seed(7)
    A = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    B = torch.randn(N, K, device=gpu, generator=g).bfloat16()
    # (native GEMM contract: leading dimensions are multiples of 8 elements)
    a = A.t().contiguous() if ak else A
    b = B.t().contiguous() if bk else B
    C = torch.empty(M, N, device=gpu)
    big_tiles(tile)
    NN.lib().gemm(a.data_ptr(), M if ak else K, ak, b.data_ptr(), N if bk else K, bk, C.data_ptr(), N, M, N, K, 1.0,
                  0.0, 0, 0, 1, 1, 1, 0, 0, 0, NN.stream())
    ref = A.float() @ B.float().t()
    assert rel_err(C, ref) < 1e-5


def test_conv_bias_relu_fused(gpu):
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(4)
    x = bf(torch.randn(2, 16, 10, 10, generator=g)).float()
    w = bf(torch.randn(24, 16, 3, 3, generator=g) * 0.1).float()
    b = torch.randn(24, generator=g)
    y = F.conv2d_fwd(x.to(gpu), w.to(gpu), b.to(gpu), (1, 1), (1, 1), relu=True)
    ref = torch.relu(TF.conv2d(x, w, b, 1, 1))
    assert rel_err(y, ref) < 1e-5


# --------------------------------------------------------------- batch norm
@pytest.mark.parametrize("C", [64, 20, 256])
@pytest.mark.parametrize("relu,residual", [(False, False), (True, False), (True, True)])
def test_batchnorm(gpu, C, relu, residual):
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, C, 7, 9, generator=g) * 2 + 0.5
    gam = torch.rand(C, generator=g) + 0.5
    bet = torch.randn(C, generator=g)
    res = torch.randn(4, C, 7, 9, generator=g) if residual else None
    dy = torch.randn(4, C, 7, 9, generator=g)
    # reference
    xr = x.clone().requires_grad_(True)
    gr, br = gam.clone().requires_grad_(True), bet.clone().requires_grad_(True)
    rr = res.clone().requires_grad_(True) if residual else None
    rm, rv = torch.zeros(C), torch.ones(C)
    yr = TF.batch_norm(xr, rm, rv, gr, br, True, 0.1, 1e-5)
    if residual:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    yr.backward(dy)
    cl = lambda t: t.to(gpu).contiguous(memory_format=torch.channels_last)  # noqa: E731
    rmg, rvg = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    y, st = F.batchnorm_fwd(cl(x), gam.to(gpu), bet.to(gpu), rmg, rvg, True, 0.1, 1e-5, relu,
                            cl(res) if residual else None)
    assert rel_err(y, yr.detach()) < 1e-5
    assert rel_err(rmg, rm) < 1e-5 and rel_err(rvg, rv) < 1e-5
    dx, dg, dbt, dres = F.batchnorm_bwd(cl(x), cl(dy), gam.to(gpu), st, y if (relu and residual) else None,
                                        need_dres=residual, relu=relu)
    assert rel_err(dx, xr.grad) < 1e-4
    assert rel_err(dg, gr.grad) < 1e-4
    assert rel_err(dbt, br.grad) < 1e-4
    if residual:
        assert rel_err(dres, rr.grad) < 1e-5


def test_batchnorm_bf16(gpu):
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(6)
    C = 128
    x = bf(torch.randn(8, C, 14, 14, generator=g))
    gam, bet = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)
    rm, rv = torch.zeros(C), torch.ones(C)
    yr = torch.relu(TF.batch_norm(x.float(), rm, rv, gam, bet, True, 0.1, 1e-5))
    y, _ = F.batchnorm_fwd(x.to(gpu).contiguous(memory_format=torch.channels_last), gam.to(gpu), bet.to(gpu),
                           torch.zeros(C, device=gpu), torch.ones(C, device=gpu), True, relu=True)
    assert y.dtype == torch.bfloat16
    assert rel_err(y, yr) < 1e-2


# ------------------------------------------------------------------ pooling
@pytest.mark.parametrize("H,W", [(13, 11), (16, 16), (8, 9)])
def test_maxpool_bwd_bf16_stem_shape(gpu, H, W):
    """bf16 3x3/s2/p1 max-pool (the ResNet stem's; closed-form backward
    kernel) vs PyTorch fp32 on the same values: a permutation of distinct
    integers per plane (exact in bf16, so no ties)."""
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(3)
    N_, C = 2, 16
    x = torch.stack([torch.randperm(H * W, generator=g).float().reshape(H, W) for _ in range(N_ * C)])
    x = x.reshape(N_, C, H, W)
    xr = x.clone().requires_grad_(True)
    yr = TF.max_pool2d(xr, 3, 2, 1)
    dy = torch.randn(yr.shape, generator=g).bfloat16().float()
    yr.backward(dy)
    xg = x.to(gpu).bfloat16().contiguous(memory_format=torch.channels_last)
    y, arg = F.pool2d_fwd(xg, (3, 3), (2, 2), (1, 1), True)
    assert torch.equal(y.float().cpu(), yr.detach())
    dx = F.pool2d_bwd(xg.shape, xg, dy.to(gpu).bfloat16().contiguous(memory_format=torch.channels_last), arg,
                      (3, 3), (2, 2), (1, 1), True)
    assert rel_err(dx, xr.grad) < 5e-3


@pytest.mark.parametrize("is_max", [True, False])
@pytest.mark.parametrize("k,s,p", [(3, 2, 1), (2, 2, 0), (3, 1, 1)])
def test_pool(gpu, is_max, k, s, p):
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 16, 13, 11, generator=g)
    xr = x.clone().requires_grad_(True)
    yr = TF.max_pool2d(xr, k, s, p) if is_max else TF.avg_pool2d(xr, k, s, p, count_include_pad=True)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    xg = x.to(gpu).contiguous(memory_format=torch.channels_last)
    y, arg = F.pool2d_fwd(xg, (k, k), (s, s), (p, p), is_max)
    assert rel_err(y, yr.detach()) < 1e-6
    dx = F.pool2d_bwd(xg.shape, xg, dy.to(gpu).contiguous(memory_format=torch.channels_last), arg, (k, k), (s, s),
                      (p, p), is_max)
    assert rel_err(dx, xr.grad) < 1e-6


def test_global_avgpool(gpu):
    from singa_amd.ops import functional as F
    x = torch.randn(4, 64, 7, 7)
    y = F.global_avgpool_fwd(x.to(gpu).contiguous(memory_format=torch.channels_last))
    assert rel_err(y, x.mean((2, 3))) < 1e-6
    dy = torch.randn(4, 64)
    dx = F.global_avgpool_bwd(dy.to(gpu), x.shape)
    assert rel_err(dx, (dy[:, :, None, None] / 49).expand_as(x)) < 1e-6


@pytest.mark.parametrize("C,size,dtype", [(16, 5, torch.float32), (12, 5, torch.float32), (64, 5, torch.bfloat16),
                                           (96, 5, torch.float32), (256, 3, torch.bfloat16), (192, 5, torch.bfloat16)])
def test_lrn(gpu, C, size, dtype):
    """LRN forward/backward (pixel-staged kernel for C % 8 == 0, the
    per-element kernel otherwise) vs torch.nn.functional.local_response_norm
    in fp32 with autograd."""
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(13)
    x = torch.randn(3, C, 7, 5, generator=g).to(dtype)
    dy = torch.randn(3, C, 7, 5, generator=g).to(dtype)
    xr = x.float().requires_grad_(True)
    tref = TF.local_response_norm(xr, size, 1e-2, 0.75, 2.0)
    tref.backward(dy.float())
    cl = lambda t: t.to(gpu).contiguous(memory_format=torch.channels_last)  # noqa: E731
    y, norm = F.lrn_fwd(cl(x), size, 1e-2, 0.75, 2.0)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(y, tref.detach()) < tol
    dx = F.lrn_bwd(cl(x), cl(dy), norm, size, 1e-2, 0.75, 2.0)
    assert rel_err(dx, xr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)
    # CPU reference path of the wrappers agrees too
    y_c, norm_c = F.lrn_fwd(x.float(), size, 1e-2, 0.75, 2.0)
    assert rel_err(F.lrn_bwd(x.float(), dy.float(), norm_c, size, 1e-2, 0.75, 2.0), xr.grad) < 1e-5


# ------------------------------------------------------- softmax / losses
@pytest.mark.parametrize("C", [10, 1000, 3000])
def test_softmax_xent(gpu, C):
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(8)
    x = torch.randn(33, C, generator=g) * 3
    lab = torch.randint(0, C, (33,), generator=g)
    loss, correct, dx = F.softmax_xent(x.to(gpu), lab.to(gpu), topk=5)
    xr = x.clone().requires_grad_(True)
    l = TF.cross_entropy(xr, lab)
    l.backward()
    assert abs(float(loss.mean()) - float(l)) < 1e-5
    assert rel_err(dx, xr.grad) < 1e-5
    top5 = (x.topk(5, 1).indices == lab[:, None]).any(1).float()
    assert torch.equal(correct.cpu(), top5)
    y = F.softmax(x.to(gpu))
    assert rel_err(y, torch.softmax(x, 1)) < 1e-6
    dyy = torch.randn(33, C, generator=g)
    d = F.softmax_bwd(y, dyy.to(gpu))
    sr = torch.softmax(x, 1)
    assert rel_err(d, sr * (dyy - (dyy * sr).sum(1, keepdim=True))) < 1e-5


@pytest.mark.parametrize("R,D", [(64, 768), (4099, 768), (37, 100), (300, 1024), (50, 2048), (40, 2050), (9, 36)])
def test_layernorm(gpu, R, D):
    """fp32 kernels vs PyTorch fp32: the row-batched backward (D % 4 == 0,
    D <= 2048, partial last workgroup, padded lanes) and the per-row
    fallback (D = 2050)."""
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(9)
    x = torch.randn(R, D, generator=g)
    gm, bt = torch.rand(D, generator=g) + 0.5, torch.randn(D, generator=g)
    dy = torch.randn(R, D, generator=g)
    xr, gr, br = x.clone().requires_grad_(True), gm.clone().requires_grad_(True), bt.clone().requires_grad_(True)
    yr = TF.layer_norm(xr, (D,), gr, br, 1e-5)
    yr.backward(dy)
    y, mu, rs = F.layernorm_fwd(x.to(gpu), gm.to(gpu), bt.to(gpu))
    assert rel_err(y, yr.detach()) < 1e-5
    dx, dg, db = F.layernorm_bwd(x.to(gpu), dy.to(gpu), gm.to(gpu), mu, rs)
    assert rel_err(dx, xr.grad) < 1e-4 and rel_err(dg, gr.grad) < 1e-4 and rel_err(db, br.grad) < 1e-4


def test_layernorm_bwd_bf16(gpu):
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(10)
    x = torch.randn(4096, 768, generator=g).bfloat16()
    gm = torch.rand(768, generator=g) + 0.5
    dy = torch.randn(4096, 768, generator=g).bfloat16()
    xr, gr = x.float().requires_grad_(True), gm.clone().requires_grad_(True)
    TF.layer_norm(xr, (768,), gr, None, 1e-5).backward(dy.float())
    _, mu, rs = F.layernorm_fwd(x.to(gpu), gm.to(gpu), None)
    dx, dg, db = F.layernorm_bwd(x.to(gpu), dy.to(gpu), gm.to(gpu), mu, rs)
    assert dx.dtype == torch.bfloat16
    assert rel_err(dx, xr.grad) < 1e-2 and rel_err(dg, gr.grad) < 1e-4
    assert rel_err(db, dy.float().sum(0)) < 1e-4


@pytest.mark.parametrize("C", [5, 64, 128, 300, 1024])
@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                          (torch.bfloat16, torch.bfloat16)])
def test_softmax_short_rows(gpu, C, in_dt, out_dt):
    """Wave-per-row softmax (C <= 1024) with an independent output dtype,
    and its backward, vs PyTorch fp32."""
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(2, 3, 77, C, generator=g) * 3).to(in_dt)
    y = F.softmax(x.to(gpu), -1, out_dtype=out_dt)
    ref = torch.softmax(x.float(), -1)
    assert y.dtype == out_dt and y.shape == x.shape
    assert rel_err(y, ref) < (1e-6 if out_dt == torch.float32 else 1e-2)
    dy = torch.randn(x.shape, generator=g).to(out_dt)
    d = F.softmax_bwd(y, dy.to(gpu))
    yf = y.float().cpu()
    assert rel_err(d, yf * (dy.float() - (dy.float() * yf).sum(-1, keepdim=True))) < (1e-5 if out_dt == torch.float32
                                                                                       else 2e-2)


@pytest.mark.parametrize("op", ["relu", "sigmoid", "tanh", "stanh", "gelu", "softplus", "exp", "abs", "square",
                                "leakyrelu", "elu", "selu"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_unary(gpu, op, dtype):
    from singa_amd.ops import functional as F
    x = torch.randn(1003) * 2
    alpha = 0.1 if op in ("leakyrelu",) else (1.0 if op == "elu" else 0.0)
    y_ref = F.unary(op, x.to(dtype).float(), alpha)
    y = F.unary(op, x.to(dtype).to(gpu), alpha)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(y, y_ref) < tol
    dy = torch.randn(1003)
    d_ref = F.unary_bwd(op, x.to(dtype).float(), y_ref, dy.to(dtype).float(), alpha)
    d = F.unary_bwd(op, x.to(dtype).to(gpu), y, dy.to(dtype).to(gpu), alpha)
    assert rel_err(d, d_ref) < (1e-4 if dtype == torch.float32 else 2e-2)


def test_add_relu_and_cast(gpu):
    from singa_amd.ops import functional as F
    a, b = torch.randn(4, 8, 5, 5), torch.randn(4, 8, 5, 5)
    cl = lambda t: t.to(gpu).contiguous(memory_format=torch.channels_last)  # noqa: E731
    y = F.add_act(cl(a), cl(b), relu=True)
    assert y.is_contiguous(memory_format=torch.channels_last)
    assert rel_err(y, torch.relu(a + b)) < 1e-7
    c = F.cast(cl(a), torch.bfloat16)
    assert c.dtype == torch.bfloat16 and rel_err(c, a) < 1e-2


def test_dropout(gpu):
    from singa_amd.ops import functional as F
    x = torch.ones(100000, device=gpu)
    y, mask = F.dropout_fwd(x, 0.3, 42, 0)
    keep = float(mask.float().mean())
    assert abs(keep - 0.7) < 0.01
    assert torch.allclose(y[mask.bool()], torch.full_like(y[mask.bool()], 1 / 0.7))
    dx = F.dropout_bwd(torch.ones_like(x), mask, 0.3)
    assert torch.equal(dx, y)
    y2, m2 = F.dropout_fwd(x, 0.3, 42, 0)
    assert torch.equal(mask, m2)  # reproducible per (seed, offset)
    # the 8-wide kernel (n % 8 == 0) draws exactly the scalar kernel's mask
    for dt in (torch.float32, torch.bfloat16):
        xo = torch.randn(100001, device=gpu).to(dt)
        ys, ms = F.dropout_fwd(xo, 0.3, 7, 5)
        yv, mv = F.dropout_fwd(xo[:100000].clone(), 0.3, 7, 5)
        assert torch.equal(ms[:100000], mv) and torch.equal(ys[:100000], yv)
        g = torch.randn(100000, device=gpu).to(dt)
        assert rel_err(F.dropout_bwd(g, mv, 0.3), g.float() * mv.float() / 0.7) < (1e-6 if dt == torch.float32 else 5e-3)


# ----------------------------------------------------------------- optimiser
@pytest.mark.parametrize("cls,kw", [("SGD", dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
                                    ("SGD", dict(lr=0.1, momentum=0.9, nesterov=True)),
                                    ("Adam", dict(lr=1e-3, weight_decay=1e-2)),
                                    ("AdamW", dict(lr=1e-3)),
                                    ("AdaGrad", dict(lr=0.1)), ("RMSProp", dict(lr=0.01)),
                                    ("AdaDelta", dict(lr=1.0)), ("RefSGD", dict(lr=0.1, momentum=0.9)),
                                    ("Nesterov", dict(lr=0.1, momentum=0.9))])
def test_fused_optimizer_matches_cpu(gpu, cls, kw):
    from singa_amd import opt as O
    from singa_amd.tensor import Tensor
    g = torch.Generator().manual_seed(10)
    shapes = [(64, 3, 3, 3), (64,), (200, 10)]
    init = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g) for s in shapes] for _ in range(3)]
    outs = []
    for dev in ("cpu", gpu):
        ps = []
        for i, t in enumerate(init):
            p = Tensor(data=t.clone().to(dev), stores_grad=True)
            p.param_meta = {"lr_mult": 1.0 if i != 1 else 2.0, "wd_mult": 1.0 if i != 1 else 0.0}
            ps.append(p)
        o = getattr(O, cls)(**kw)
        o.attach(ps)
        for step in grads:
            for p, gg in zip(ps, step):
                p.grad_view.copy_(gg.to(dev))
            o.update()
            o.step()
        outs.append([p.data.detach().float().cpu().clone() for p in ps])
    for a, b in zip(*outs):
        assert rel_err(b, a) < 1e-5


def test_easgd_and_rsync_kernels(gpu):
    from singa_amd.ops import native as NT
    w = torch.randn(1000, device=gpu)
    c = torch.randn(1000, device=gpu)
    w0 = w.clone()
    d = torch.empty_like(w)
    NT.lib().easgd_diff(w.data_ptr(), c.data_ptr(), d.data_ptr(), 1000, 0.25, NT.stream())
    assert rel_err(d, 0.25 * (w0 - c)) < 1e-6 and rel_err(w, w0 - 0.25 * (w0 - c)) < 1e-6
    snap = torch.randn(1000, device=gpu)
    out = torch.empty(100, device=gpu)
    NT.lib().rsync_gather(w.data_ptr(), snap.data_ptr(), out.data_ptr(), 100, 1000, 7, 13, NT.stream())
    idx = (13 + torch.arange(100) * 7) % 1000
    assert rel_err(out, (w - snap)[idx.to(gpu)]) < 1e-6


@pytest.mark.parametrize("det", [False, True])
@pytest.mark.parametrize("C,K,H", [(64, 256, 28), (128, 64, 14), (32, 1024, 7)])
def test_conv_epilogue_bn_stats(gpu, C, K, H, det):
    """BN statistics summed by the conv epilogue == the separate stats pass."""
    import singa_amd
    from singa_amd.ops import functional as F
    singa_amd.set_deterministic(det)
    g = torch.Generator(device=gpu).manual_seed(1)
    x = torch.randn(8, C, H, H, device=gpu, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 3, 3, device=gpu, generator=g) * 0.05).bfloat16().contiguous(
        memory_format=torch.channels_last)
    y1 = F.conv2d_fwd(x, w, None, (1, 1), (1, 1), out_dtype=torch.bfloat16, bn_stats=True)
    assert getattr(y1, "_sg_bn_ws", None) is not None
    y2 = F.conv2d_fwd(x, w, None, (1, 1), (1, 1), out_dtype=torch.bfloat16)
    assert torch.equal(y1, y2)
    gam = torch.rand(K, device=gpu) + 0.5
    bet = torch.randn(K, device=gpu)
    outs = []
    for y in (y1, y2):
        rm, rv = torch.zeros(K, device=gpu), torch.ones(K, device=gpu)
        out, st = F.batchnorm_fwd(y, gam, bet, rm, rv, True, 0.1, 1e-5, relu=True)
        outs.append((out.float(), st.mean.clone(), st.invstd.clone(), rm, rv))
    singa_amd.set_deterministic(False)
    for a, b in zip(outs[0], outs[1]):
        assert rel_err(a, b) < 1e-4


@pytest.mark.parametrize("C,K,H,R,st", [(64, 256, 56, 1, 1), (128, 128, 28, 3, 1), (256, 64, 56, 1, 1),
                                         (512, 512, 7, 3, 1), (256, 512, 56, 1, 2)])
def test_conv_bitwise_deterministic(gpu, C, K, H, R, st):
    """Repeated launches with allocator churn in between give bit-identical
    outputs (fwd with/without fused BN stats, dgrad)."""
    from singa_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(3)
    x = torch.randn(32, C, H, H, device=gpu, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device=gpu, generator=g) * 0.05).bfloat16().contiguous(
        memory_format=torch.channels_last)
    pad = R // 2
    ref = F.conv2d_fwd(x, w, None, (st, st), (pad, pad), out_dtype=torch.bfloat16)
    dy = torch.randn(ref.shape, device=gpu, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    dref = F.conv2d_bwd(x, w, dy, (st, st), (pad, pad), need_dx=True)[0]
    junk = []
    for i in range(12):
        junk.append(torch.randn(int(1e6) * (1 + i % 3), device=gpu))
        if i % 4 == 3:
            junk.clear()
        y = F.conv2d_fwd(x, w, None, (st, st), (pad, pad), out_dtype=torch.bfloat16, bn_stats=bool(i % 2))
        assert torch.equal(y, ref), i
        d = F.conv2d_bwd(x, w, dy, (st, st), (pad, pad), need_dx=True)[0]
        assert torch.equal(d, dref), i


@pytest.mark.parametrize("C,H", [(64, 56), (256, 14), (2048, 7)])
def test_batchnorm_bitwise_deterministic(gpu, C, H):
    import singa_amd
    from singa_amd.ops import functional as F
    singa_amd.set_deterministic(True)
    g = torch.Generator(device=gpu).manual_seed(4)
    x = (torch.randn(64, C, H, H, device=gpu, generator=g) * 3 + 1).bfloat16().contiguous(
        memory_format=torch.channels_last)
    gam, bet = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu)
    outs = []
    for _ in range(6):
        y, st = F.batchnorm_fwd(x, gam, bet, torch.zeros(C, device=gpu), torch.ones(C, device=gpu), True, 0.1, 1e-5,
                                relu=True)
        outs.append((y, st.mean.clone(), st.invstd.clone()))
    singa_amd.set_deterministic(False)
    for o in outs[1:]:
        assert torch.equal(o[1], outs[0][1]) and torch.equal(o[2], outs[0][2])
        assert torch.equal(o[0], outs[0][0])


def _guarded(n, dtype, gpu, pad=4096):
    """A view of n elements inside a buffer with `pad` sentinel elements on
    both sides; returns (view, check) where check() asserts the guards."""
    buf = torch.full((n + 2 * pad,), 7.0, dtype=dtype, device=gpu)
    view = buf[pad:pad + n]

    def check(tag):
        torch.cuda.synchronize()
        assert bool((buf[:pad] == 7.0).all()), f"{tag}: write before the buffer"
        assert bool((buf[pad + n:] == 7.0).all()), f"{tag}: write past the buffer"
    return view, check


@pytest.mark.parametrize("Nb,C,K,H,R,st", [(3, 64, 256, 14, 1, 1), (2, 128, 128, 15, 3, 2), (2, 96, 40, 9, 3, 1),
                                           (4, 256, 64, 7, 1, 2), (2, 8, 64, 33, 7, 2)])
def test_conv_kernels_stay_in_bounds(gpu, Nb, C, K, H, R, st):
    from singa_amd.ops import native as NN
    L = NN.lib()
    pad = R // 2
    Ho = (H + 2 * pad - R) // st + 1
    g = torch.Generator(device=gpu).manual_seed(9)
    x = torch.randn(Nb * H * H * C, device=gpu, generator=g).bfloat16()
    w = (torch.randn(K * R * R * C, device=gpu, generator=g) * 0.05).bfloat16()
    dy = torch.randn(Nb * Ho * Ho * K, device=gpu, generator=g).bfloat16()
    s = NN.stream()
    for stats in (False, True):
        y, chk = _guarded(Nb * Ho * Ho * K, torch.bfloat16, gpu)
        ws = None
        if stats:
            rows = L.conv_stats_rows(Nb * Ho * Ho, K)
            ws, wchk = _guarded(max(rows, 1) * 2 * K, torch.float32, gpu)
            ws.zero_()
        L.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, Nb, H, H, C, K, R, R, Ho, Ho, st, st, pad, pad, 1, 1,
                   0, 0, s, ws.data_ptr() if ws is not None else 0)
        chk("conv_fwd")
        if ws is not None:
            wchk("conv_fwd stats")
    if st * st <= 16:
        dx, chk = _guarded(Nb * H * H * C, torch.bfloat16, gpu)
        L.conv_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), Nb, H, H, C, K, R, R, Ho, Ho, st, st, pad, pad, 1, 1, 0,
                     s)
        chk("conv_dgrad")
    dw, chk = _guarded(K * R * R * C, torch.float32, gpu)
    dw.zero_()
    L.conv_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), Nb, H, H, C, K, R, R, Ho, Ho, st, st, pad, pad, 1, 1, 0, s)
    chk("conv_wgrad")


@pytest.mark.parametrize("R,C", [(1000, 64), (37, 256), (4096, 24)])
def test_bn_kernels_stay_in_bounds(gpu, R, C):
    from singa_amd.ops import native as NN
    L = NN.lib()
    s = NN.stream()
    g = torch.Generator(device=gpu).manual_seed(10)
    x = torch.randn(R * C, device=gpu, generator=g).bfloat16()
    dy = torch.randn(R * C, device=gpu, generator=g).bfloat16()
    f = lambda: torch.rand(C, device=gpu) + 0.5  # noqa: E731
    gam, bet, rm, rv = f(), f(), torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    p = [torch.empty(C, device=gpu) for _ in range(4)]
    ws, wchk = _guarded(L.colreduce_ws(R, C), torch.float32, gpu)
    L.bn_fwd_stats(x.data_ptr(), ws.data_ptr(), gam.data_ptr(), bet.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                   *[t.data_ptr() for t in p], R, C, 0.1, 1e-5, NN.BF16, s)
    wchk("bn_fwd_stats ws")
    y, chk = _guarded(R * C, torch.bfloat16, gpu)
    L.bn_apply(x.data_ptr(), p[2].data_ptr(), p[3].data_ptr(), 0, y.data_ptr(), R, C, 1, NN.BF16, s, 0)
    chk("bn_apply")
    coef = torch.empty(3 * C, device=gpu)
    dg, db = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
    dx, chk2 = _guarded(R * C, torch.bfloat16, gpu)
    dres, chk3 = _guarded(R * C, torch.bfloat16, gpu)
    L.bn_bwd(x.data_ptr(), dy.data_ptr(), y.data_ptr(), p[2].data_ptr(), p[3].data_ptr(), p[0].data_ptr(),
             p[1].data_ptr(), gam.data_ptr(), ws.data_ptr(), coef.data_ptr(), dg.data_ptr(), db.data_ptr(),
             dx.data_ptr(), dres.data_ptr(), R, C, 1, NN.BF16, s)
    wchk("bn_bwd ws")
    chk2("bn_bwd dx")
    chk3("bn_bwd dres")


def test_fused_bn_stats_under_graph_replay(gpu):
    """conv (+epilogue BN statistics) -> BN, captured once and replayed: every
    replay must see freshly zeroed statistics (the same outputs: the slot-row
    atomics may sum in another order, so a few bf16 outputs can move by one
    ulp; statistics that were not re-zeroed would double the sums)."""
    from singa_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(11)
    x = torch.randn(8, 64, 28, 28, device=gpu, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(128, 64, 3, 3, device=gpu, generator=g) * 0.05).bfloat16().contiguous(
        memory_format=torch.channels_last)
    gam, bet = torch.rand(128, device=gpu) + 0.5, torch.randn(128, device=gpu)
    rm, rv = torch.zeros(128, device=gpu), torch.ones(128, device=gpu)

    def step():
        y = F.conv2d_fwd(x, w, None, (1, 1), (1, 1), out_dtype=torch.bfloat16, bn_stats=True)
        out, st = F.batchnorm_fwd(y, gam, bet, rm, rv, True, 0.1, 1e-5, relu=True)
        return out, st.mean, st.invstd

    ref = [t.clone() for t in step()]
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        outs = step()
    for _ in range(4):
        gr.replay()
        torch.cuda.synchronize()
        for a, b in zip(outs, ref):
            assert rel_err(a, b) < 1e-4


@pytest.mark.parametrize("bn", [False, True])
@pytest.mark.parametrize("C,K,H,st", [(64, 256, 64, 1), (64, 128, 96, 1), (256, 64, 64, 1), (64, 256, 96, 2),
                                     (512, 128, 96, 1)])
def test_conv_short_k_single_stage(gpu, C, K, H, st, bn):
    """The single-stage short-K GEMM variant (tuning knob 6: four workgroups
    per CU, bf16-staged epilogue) on 1x1 convs big enough to take it: forward
    (with and without the fused BN statistics) and data gradient == the
    2-stage kernels' results and a PyTorch fp32 reference."""
    from singa_amd.ops import functional as F
    from singa_amd.ops import native as NN
    g = torch.Generator(device=gpu).manual_seed(5)
    Nb = 16
    x = torch.randn(Nb, C, H, H, device=gpu, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 1, 1, device=gpu, generator=g) * 0.1).bfloat16().contiguous(
        memory_format=torch.channels_last)
    Ho = (H - 1) // st + 1
    dy = torch.randn(Nb, K, Ho, Ho, device=gpu, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    outs = {}
    try:
        for knob in (0, 8):
            NN.lib().set_tuning(6, knob)
            y = F.conv2d_fwd(x, w, None, (st, st), (0, 0), out_dtype=torch.bfloat16, bn_stats=bn)
            dx = F.conv2d_bwd(x, w, dy, (st, st), (0, 0), need_dx=True)[0]
            ws = getattr(y, "_sg_bn_ws", None)
            outs[knob] = (y.float(), dx.float(), None if ws is None else ws[0][: 2 * K * ws[1]].view(ws[1], 2, K).sum(0))
    finally:
        NN.lib().set_tuning(6, 2)  # the default
    ref = TF.conv2d(x.float(), w.float(), stride=st)
    dref = TF.conv_transpose2d(dy.float(), w.float(), stride=st, output_padding=(H - 1) % st if st > 1 else 0)
    for knob in (0, 8):
        yk, dxk, wsk = outs[knob]
        assert rel_err(yk, ref) < 1e-2
        assert rel_err(dxk, dref) < 1e-2
    assert torch.equal(outs[0][0], outs[8][0])  # same bf16 rounding of the same fp32 sums
    assert torch.equal(outs[0][1], outs[8][1])
    if bn:
        yb = outs[0][0]
        s = torch.stack([yb.sum((0, 2, 3)), (yb * yb).sum((0, 2, 3))])
        assert rel_err(outs[8][2], s) < 1e-4 and rel_err(outs[0][2], s) < 1e-4


@pytest.mark.parametrize("B,S,H,D,masked", [(2, 64, 4, 64, False), (3, 128, 12, 64, True), (1, 40, 2, 32, False)])
def test_attention_qkv_in_place_heads(gpu, B, S, H, D, masked):
    """attention_qkv_fwd / _bwd (two-level-batch MFMA GEMMs addressing the
    heads inside the [B, S, 3, H, D] projection) vs PyTorch fp32 multi-head
    attention on the same bf16 inputs."""
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(12)
    qkv = (torch.randn(B, S, 3 * H * D, generator=g) * 0.5).bfloat16()
    do = torch.randn(B, S, H * D, generator=g).bfloat16()
    mask = ((torch.rand(B, 1, 1, S, generator=g) > 0.8).float() * -10000.0) if masked else None
    o, p = F.attention_qkv_fwd(qkv.to(gpu), H, mask.to(gpu) if masked else None)
    dqkv = F.attention_qkv_bwd(qkv.to(gpu), p, do.to(gpu), H)
    x = qkv.float().requires_grad_(True)
    t = x.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
    s = t[0] @ t[1].transpose(-1, -2) / math.sqrt(D)
    if masked:
        s = s + mask
    ref = (torch.softmax(s, -1) @ t[2]).permute(0, 2, 1, 3).reshape(B, S, H * D)
    ref.backward(do.float())
    assert o.shape == (B, S, H * D) and dqkv.shape == qkv.shape
    assert rel_err(o, ref.detach()) < 2e-2
    assert rel_err(dqkv, x.grad) < 3e-2


@pytest.mark.parametrize("R,C,dtype", [(4096, 768, torch.bfloat16), (1000, 3072, torch.bfloat16), (37, 8, torch.float32),
                                       (5000, 2048, torch.float32), (300, 100, torch.bfloat16),
                                       (4096, 2304, torch.bfloat16), (33, 1032, torch.float32),
                                       (70, 8192, torch.bfloat16), (50, 9000, torch.bfloat16)])
def test_colsum_accumulate(gpu, R, C, dtype):
    """Column sums accumulated into an existing fp32 buffer (the bias-gradient
    path: one launch for C % 8 == 0, C <= 2048; the workspace + finalize
    reduction otherwise) and the fresh-output path, vs PyTorch fp32."""
    from singa_amd.ops import functional as F
    g = torch.Generator().manual_seed(14)
    x = torch.randn(R, C, generator=g).to(dtype)
    base = torch.randn(C, generator=g)
    out = base.clone().to(gpu)
    r, _ = F.colsum(x.to(gpu), out=out)
    ref = base + x.float().sum(0)
    assert r.data_ptr() == out.data_ptr()
    assert rel_err(out, ref) < 1e-5
    fresh, sq = F.colsum(x.to(gpu), with_sq=True)
    assert rel_err(fresh, x.float().sum(0)) < 1e-5 and rel_err(sq, (x.float() ** 2).sum(0)) < 1e-5


@pytest.mark.parametrize("M,K,N", [(262145, 64, 128), (131075, 72, 256), (270000, 128, 128)])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_gemm_persistent_short_k(gpu, M, K, N, beta):
    """The persistent short-K kernel (knob 9: B resident in LDS, M-tiles walked
    with a two-slot A ring, counted waits, buffer stores for the ragged last
    tile) against fp32 torch, plain and accumulating (beta)."""
    from singa_amd.ops import functional as F
    from singa_amd.ops import native as NN
    g = torch.Generator(device=gpu).manual_seed(11)
    x = torch.randn(M, K, device=gpu, generator=g).bfloat16()
    w = torch.randn(N, K, device=gpu, generator=g).bfloat16()
    c0 = torch.randn(M, N, device=gpu, generator=g).bfloat16()
    c = c0.clone()
    NN.lib().set_tuning(9, 1)
    try:
        F.gemm(x, w, tb=True, out=c, beta=beta)
    finally:
        NN.lib().set_tuning(9, 1)  # (the default: knob 9 is on)
    ref = x.float() @ w.float().t() + beta * c0.float()
    assert rel_err(c, ref) < 5e-3
    assert rel_err(c[-5:], ref[-5:]) < 5e-3  # the partial last M-tile


def test_conv1x1_persistent_short_k_bn_stats(gpu):
    """1x1 conv forward through the persistent kernel with the fused BN
    statistics (kept in registers across the workgroup's tiles) equals the
    default kernel's output and batch statistics."""
    from singa_amd.ops import functional as F
    from singa_amd.ops import native as NN
    g = torch.Generator(device=gpu).manual_seed(3)
    x = torch.randn(64, 64, 56, 56, device=gpu, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(256, 64, 1, 1, device=gpu, generator=g) * 0.1).bfloat16().contiguous(
        memory_format=torch.channels_last)
    res = []
    for knob in (0, 1):
        NN.lib().set_tuning(9, knob)
        try:
            y = F.conv2d_fwd(x, w, None, (1, 1), (0, 0), out_dtype=torch.bfloat16, bn_stats=True)
            gam, bet = torch.ones(256, device=gpu), torch.zeros(256, device=gpu)
            rm, rv = torch.zeros(256, device=gpu), torch.ones(256, device=gpu)
            _, st = F.batchnorm_fwd(y, gam, bet, rm, rv, True, 0.1, 1e-5, relu=True)
            res.append((y.float(), st.mean.clone(), st.invstd.clone()))
        finally:
            NN.lib().set_tuning(9, 1)  # (the default)
    for a, b in zip(res[1], res[0]):
        assert rel_err(a, b) < 1e-4
