"""CppCPU compute backend: dispatch of host (CPU) tensors to the native C++
kernels of ``_core.cpu`` (csrc/runtime/cpu_ops.cc).

The reference's CPU device evaluates every layer with mshadow's CPU
expression loops and a BLAS sgemm (include/mshadow/tensor_cpu-inl.hpp:52-165,
src/worker/layer.cc:18-764).  Here the ``CppCPU`` device runs its compute on
this framework's own C++ kernels (a persistent worker pool, packed AVX2/FMA
GEMM, im2col convolution, pooling, LRN, softmax-xent, normalisation,
elementwise / broadcast / reduction loops); PyTorch only owns the host
storage and its free views.

PyTorch's CPU ops remain the numerics ORACLE of the tests:
``with torch_oracle():`` (or ``SINGA_AMD_CPU=torch``) routes the same
functional calls to the plain PyTorch expressions instead.
"""
from __future__ import annotations

import contextlib
import importlib
import os
from typing import Optional

import torch

_mod = None
_tried = False
_ORACLE = 0

# dtype codes shared with cpu_ops.h (f16 has no host conversion: never native)
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.int32: 3, torch.int64: 4, torch.uint8: 5, torch.float64: 6}


def lib():
    """``_core.cpu`` or None (runtime not built)."""
    global _mod, _tried
    if not _tried:
        _tried = True
        try:
            _mod = getattr(importlib.import_module("singa_amd._core"), "cpu", None)
        except Exception:  # pragma: no cover - reported by the build check
            _mod = None
    return _mod


def enabled() -> bool:
    """Native CPU compute is on (default) -- off inside :func:`torch_oracle`."""
    return _ORACLE == 0 and os.environ.get("SINGA_AMD_CPU", "native") != "torch" and lib() is not None


@contextlib.contextmanager
def torch_oracle():
    """Run host ops on the PyTorch reference expressions (the test oracle)."""
    global _ORACLE
    _ORACLE += 1
    try:
        yield
    finally:
        _ORACLE -= 1


def ok(*ts) -> bool:
    """Compute ops: every operand an fp32 host tensor (None allowed)."""
    if not enabled():
        return False
    for t in ts:
        if t is not None and (t.is_cuda or t.dtype != torch.float32):
            return False
    return True


def copy_ok(*ts) -> bool:
    """Copy / fill ops: host tensors of a dtype with a native conversion."""
    if not enabled():
        return False
    return all(t is None or (not t.is_cuda and t.dtype in _DT) for t in ts)


def dt(t: torch.Tensor) -> int:
    return _DT[t.dtype]


def p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def dense32(t: torch.Tensor) -> torch.Tensor:
    """Row-major dense fp32 (one native copy if it is not)."""
    if t.dtype == torch.float32 and t.is_contiguous():
        return t
    out = torch.empty(t.shape, dtype=torch.float32)
    from . import glue as G
    return G.copy_(out, t)


# ------------------------------------------------------------------ kernels
def gemm(a: torch.Tensor, lda: int, a_kouter: bool, b: torch.Tensor, ldb: int, b_kouter: bool, out: torch.Tensor,
         M: int, Nn: int, K: int, alpha: float, beta: float, bias: Optional[torch.Tensor], relu: bool,
         batch: int = 1, sa: int = 0, sb: int = 0, sc: int = 0) -> None:
    """out[M][Nn] (row-major, ld Nn) = alpha op(a) op(b) + beta out (+ bias) (relu).
    ``a_kouter``: a stored [K][M] (else [M][K]); ``b_kouter``: b stored [K][Nn]
    (else [Nn][K]) -- the convention of functional._mat."""
    L = lib()
    if batch == 1:
        L.gemm(bool(a_kouter), not b_kouter, M, Nn, K, float(alpha), a.data_ptr(), lda, b.data_ptr(), ldb,
               float(beta), out.data_ptr(), Nn, p(bias), bool(relu))
        return
    if bias is not None or relu:
        raise ValueError("cpu gemm: batched GEMM has no epilogue")
    L.gemm_batched(bool(a_kouter), not b_kouter, M, Nn, K, float(alpha), a.data_ptr(), lda, sa, b.data_ptr(), ldb, sb,
                   float(beta), out.data_ptr(), Nn, sc, batch)
