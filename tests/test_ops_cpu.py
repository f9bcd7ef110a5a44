"""Host-path semantics of functional ops that the GPU tests pin against the
fused kernels."""
import torch

from singa_amd.ops import functional as F


def test_gemm_colsum_c_host_path():
    """gemm_nt(..., act_grad, colsum_c): the output is the act-grad GEMM's,
    and colsum_c accumulates that output's column sums."""
    g = torch.Generator().manual_seed(0)
    dy = torch.randn(37, 24, generator=g)
    w = torch.randn(40, 24, generator=g) * 0.1
    z = torch.randn(37, 40, generator=g)
    ref = F.gemm_nt(dy, w, act_grad=("gelu", z))
    cs0 = torch.randn(40, generator=g)
    cs = cs0.clone()
    out = F.gemm_nt(dy, w, act_grad=("gelu", z), colsum_c=cs)
    torch.testing.assert_close(out, ref)
    torch.testing.assert_close(cs, cs0 + out.sum(0), rtol=1e-5, atol=1e-5)


def test_gemm_colsum_c_needs_act_grad():
    a, b = torch.randn(4, 3), torch.randn(5, 3)
    try:
        F.gemm_nt(a, b, colsum_c=torch.zeros(5))
    except ValueError:
        return
    raise AssertionError("colsum_c without act_grad must be refused")
