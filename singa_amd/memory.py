"""Framework-owned memory: tensors whose storage comes from singa_amd's own
pools (``csrc/mem/pool.cpp``) instead of PyTorch's allocator.

Reference counterparts: mshadow ``AllocSpace`` / ``FreeSpace``
(include/mshadow/tensor.h:206-385) and the ``Blob`` / ``SyncedMemory`` pair
(src/utils/blob.cc:83-298) that owned every parameter buffer.  Here the
persistent buffers -- the flat parameter store (weights, gradients, bf16
compute copy, optimiser state) -- are allocated from

* a caching HBM pool per GPU (size classes, stream-ordered reuse via events),
* a 64-byte-aligned host pool (CppCPU) or a pinned host pool (staging),

and handed to PyTorch as DLPack tensors: PyTorch supplies views and
metadata, the pool owns the bytes and gets them back when the last view
dies.  ``SINGA_AMD_NATIVE_MEM=0`` falls back to PyTorch's allocator.
"""
from __future__ import annotations

import os
from typing import Sequence

import torch

# DLPack type codes (kDLInt 0, kDLUInt 1, kDLFloat 2, kDLBfloat 4, kDLBool 6)
_CODES = {torch.float32: (2, 32), torch.float64: (2, 64), torch.float16: (2, 16), torch.bfloat16: (4, 16),
          torch.int32: (0, 32), torch.int64: (0, 64), torch.int16: (0, 16), torch.int8: (0, 8),
          torch.uint8: (1, 8), torch.bool: (6, 8)}
_DL_DEV = None


def _mod():
    from .ops import native as N
    if not N.available():
        return None
    return getattr(N.lib(), "mem", None)


def enabled() -> bool:
    return os.environ.get("SINGA_AMD_NATIVE_MEM", "1") != "0" and _mod() is not None


def _dl_device_type() -> int:
    """The DLPack device type this PyTorch build uses for GPU tensors (kDLROCM
    on ROCm builds), read from a tensor it exports."""
    global _DL_DEV
    if _DL_DEV is None:
        cap = torch.utils.dlpack.to_dlpack(torch.empty(1, device="cuda"))
        _DL_DEV = int(_mod().dl_device_type(cap))
    return _DL_DEV


def empty(shape: Sequence[int], dtype=torch.float32, device="cpu", pinned: bool = False) -> torch.Tensor:
    """A dense tensor whose storage is a block of the native pool."""
    dev = torch.device(device)
    shape = [int(s) for s in shape]
    M = _mod()
    if M is None or dtype not in _CODES or os.environ.get("SINGA_AMD_NATIVE_MEM", "1") == "0":
        return torch.empty(shape, dtype=dtype, device=dev, pin_memory=pinned and dev.type == "cpu")
    code, bits = _CODES[dtype]
    if dev.type == "cuda":
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        stream = torch.cuda.current_stream(idx).cuda_stream
        cap = M.empty(shape, code, bits, 0, idx, _dl_device_type(), stream)
    else:
        cap = M.empty(shape, code, bits, 2 if pinned else 1, 0, 1, 0)
    t = torch.utils.dlpack.from_dlpack(cap)
    return t.view(torch.bool) if dtype == torch.bool and t.dtype != torch.bool else t


def zeros(shape: Sequence[int], dtype=torch.float32, device="cpu") -> torch.Tensor:
    from .ops import glue as G
    return G.zero_(empty(shape, dtype, device))


def stats(device=None) -> dict:
    """Pool counters: allocations, cache hits, bytes in use / reserved / peak."""
    M = _mod()
    if M is None:
        return {}
    dev = torch.device(device) if device is not None else None
    if dev is not None and dev.type == "cuda":
        return dict(M.device_stats(dev.index if dev.index is not None else torch.cuda.current_device()))
    return dict(M.host_stats(False))


def empty_cache(device=None) -> None:
    """Return the pool's cached (free) blocks to the driver / OS."""
    M = _mod()
    if M is None:
        return
    dev = torch.device(device) if device is not None else None
    if dev is not None and dev.type == "cuda":
        M.empty_cache(dev.index if dev.index is not None else torch.cuda.current_device())
    else:
        M.empty_host_cache(False)
        M.empty_host_cache(True)
