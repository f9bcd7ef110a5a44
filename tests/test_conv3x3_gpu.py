"""The persistent 3x3 / stride-1 / pad-1, 64->64-channel, 56-wide convolution
(csrc/kernels/conv3x3.hip) against a PyTorch fp32 convolution and against the
generic implicit-GEMM path it replaces (``conv3x3_set(0)``): forward output and
fused BatchNorm statistics, data gradient with and without the identity-sum
BN backward's masked gradient sum."""
import pytest
import torch

from singa_amd.ops import native as N

pytestmark = pytest.mark.gpu


def _setup(gpu, n, h, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, h, 56, 64, generator=g).to(gpu).bfloat16()  # NHWC
    w = (torch.randn(64, 3, 3, 64, generator=g) * 0.05).to(gpu).bfloat16()  # [K][R][S][C]
    return x, w


def _fwd(L, x, w, on):
    n, h = x.shape[0], x.shape[1]
    L.conv3x3_set(on)
    try:
        y = torch.empty_like(x)
        ws = torch.zeros(32 * 2 * 64, dtype=torch.float32, device=x.device)
        L.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, n, h, 56, 64, 64, 3, 3, h, 56, 1, 1, 1, 1, 1, 1, 0, 0,
                   N.stream(), ws.data_ptr())
        torch.cuda.synchronize()
    finally:
        L.conv3x3_set(1)
    return y.float(), ws.view(32, 2, 64).sum(0)


def _dgrad(L, dy, w, mask, on):
    n, h = dy.shape[0], dy.shape[1]
    L.conv3x3_set(on)
    try:
        dx = torch.empty_like(dy)
        wt = torch.empty(64 * 64 * 9, dtype=torch.bfloat16, device=dy.device)
        ws = torch.zeros(32 * 2 * 64, dtype=torch.float32, device=dy.device)
        if mask is None:
            L.conv_dgrad_acc(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), n, h, 56, 64, 64, 3, 3, h, 56, 1, 1, 1, 1, 1,
                             1, 0, 0.0, N.stream(), wt.data_ptr())
        else:
            L.conv_dgrad_bn(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), n, h, 56, 64, 64, 3, 3, h, 56, 1, 1, 1, 1, 1,
                            1, wt.data_ptr(), ws.data_ptr(), 0, 0, 0, 0, 0, N.stream(), 0.0, mask.data_ptr())
        torch.cuda.synchronize()
    finally:
        L.conv3x3_set(1)
    return dx.float(), ws.view(32, 2, 64).sum(0)


@pytest.mark.parametrize("n,h", [(3, 56), (2, 16), (1, 12)])
def test_conv3x3_forward_matches_torch_and_generic(gpu, n, h):
    L = N.lib()
    x, w = _setup(gpu, n, h)
    y1, s1 = _fwd(L, x, w, 1)
    y0, s0 = _fwd(L, x, w, 0)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), padding=1)
    ref = ref.permute(0, 2, 3, 1)
    scale = float(ref.abs().max())
    assert float((y1 - ref).abs().max()) <= 1e-2 * scale
    assert float((y1 - y0).abs().max()) <= 1e-2 * scale
    # fused statistics: sums of the bf16 output
    t = y1.reshape(-1, 64)
    assert torch.allclose(s1[0], t.sum(0), rtol=1e-3, atol=1e-2 * scale)
    assert torch.allclose(s1[1], (t * t).sum(0), rtol=1e-3, atol=1e-2 * scale * scale)
    assert torch.allclose(s1, s0, rtol=2e-3, atol=2e-2 * scale * scale)


@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("n,h", [(3, 56), (2, 16)])
def test_conv3x3_data_gradient_matches_torch_and_generic(gpu, n, h, masked):
    L = N.lib()
    dy, w = _setup(gpu, n, h, seed=1)
    g = torch.Generator().manual_seed(2)
    mask = torch.randint(0, 256, (n * h * 56 * 8,), generator=g, dtype=torch.uint8).to(gpu) if masked else None
    dx1, s1 = _dgrad(L, dy, w, mask, 1)
    dx0, s0 = _dgrad(L, dy, w, mask, 0)
    ref = torch.nn.functional.conv_transpose2d(dy.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(),
                                               padding=1).permute(0, 2, 3, 1)
    scale = float(ref.abs().max())
    assert float((dx1 - ref).abs().max()) <= 1e-2 * scale
    assert float((dx1 - dx0).abs().max()) <= 1e-2 * scale
    if masked:
        bits = ((mask.view(-1, 8, 1).int() >> torch.arange(8, device=gpu).view(1, 1, 8)) & 1).view(-1, 64).float()
        want = (dx1.reshape(-1, 64) * bits).sum(0)
        assert torch.allclose(s1[0], want, rtol=1e-3, atol=1e-2 * scale)
        assert torch.allclose(s1[0], s0[0], rtol=2e-3, atol=2e-2 * scale)
        assert float(s1[1].abs().max()) == 0.0  # the masked-sum mode has no second sum
