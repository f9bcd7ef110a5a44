"""Persistent streaming GEMM (igemm_kern.h st_gemm_k, tuning knob 18) for
the 1x1-conv shapes with K >= 256: bf16 output against an fp32 PyTorch
matmul of the same operands, bitwise against the generic igemm_k path it
replaces (same MFMA k-order, one fp32 -> bf16 rounding), and its fused BN
statistics against fp32 column sums of its own bf16 output."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def knob(gpu):
    from singa_amd.ops import native as N

    L = N.lib()
    old = L.get_tuning(18)
    yield L
    L.set_tuning(18, old)


@pytest.mark.parametrize("M,N,K", [(65536 + 50, 512, 256), (32768 + 5, 1024, 512), (16384, 2048, 1024),
                                   (262144, 128, 2048)])
def test_streaming_gemm_matches_fp32_and_generic(gpu, knob, M, N, K):
    from singa_amd.ops import functional as F

    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    a = (torch.randn(M, K, device=gpu, generator=g) * 0.1).bfloat16()
    b = (torch.randn(N, K, device=gpu, generator=g) * 0.1).bfloat16()
    knob.set_tuning(18, 0)
    ref_gen = F.gemm_nt(a, b, out_dtype=torch.bfloat16)
    knob.set_tuning(18, 2)
    y = F.gemm_nt(a, b, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t()
    rel = float((y.float() - ref).norm() / ref.norm())
    assert rel < 5e-3, rel
    assert torch.equal(y, ref_gen)  # bitwise the generic kernel's result


@pytest.mark.parametrize("shape", [(32, 256, 56, 1024), (256, 512, 28, 256), (256, 1024, 14, 2048)])
def test_streaming_conv1x1_bn_stats(gpu, knob, shape):
    """1x1 conv forward with the fused BN statistics: output and per-channel
    (sum, sum of squares) equal the generic kernel's, and the sums match
    fp32 sums of the bf16 output."""
    from singa_amd.ops import functional as F

    n, c, h, k = shape
    g = torch.Generator(device=gpu).manual_seed(n * c + k)
    x = (torch.randn(n, c, h, h, device=gpu, generator=g)).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(k, c, 1, 1, device=gpu, generator=g) * (1.0 / c ** 0.5)).bfloat16()
    res = {}
    for on in (0, 1):
        knob.set_tuning(18, 2 * on)
        y = F.conv2d_fwd(x, w, None, (1, 1), (0, 0), bn_stats=True)
        ws, rows = y._sg_bn_ws
        torch.cuda.synchronize()
        st = ws.reshape(-1)[: rows * 2 * k].view(rows, 2, k).sum(0)
        res[on] = (y.clone(), st.clone())
    assert torch.equal(res[0][0], res[1][0])
    yf = res[1][0].float().permute(0, 2, 3, 1).reshape(-1, k)
    torch.testing.assert_close(res[1][1][0], yf.sum(0), rtol=2e-4, atol=2e-2)
    torch.testing.assert_close(res[1][1][1], (yf * yf).sum(0), rtol=2e-4, atol=2e-2)
    torch.testing.assert_close(res[1][1], res[0][1], rtol=2e-4, atol=2e-2)


def test_streaming_gemm_in_graph_with_generic(gpu, knob):
    """Captured into a HIP graph next to other persistent kernels and
    replayed: the queue slots come from the capture's arena, results exact."""
    from singa_amd.ops import functional as F
    from singa_amd.stream import StepGraph

    knob.set_tuning(18, 2)
    g = torch.Generator(device=gpu).manual_seed(3)
    a = (torch.randn(65536, 256, device=gpu, generator=g) * 0.1).bfloat16()
    b = (torch.randn(1024, 256, device=gpu, generator=g) * 0.1).bfloat16()
    ref = F.gemm_nt(a, b, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    box = {}
    sg = StepGraph()
    sg.capture(lambda: box.setdefault("y", F.gemm_nt(a, b, out_dtype=torch.bfloat16)))
    assert sg.queue_slots == 1
    for _ in range(3):
        box["y"].fill_(float("nan"))
        sg.replay()
        torch.cuda.synchronize()
        assert torch.equal(box["y"], ref)
    sg.release()
