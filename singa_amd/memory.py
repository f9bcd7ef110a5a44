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


class SyncedBlob:
    """Host/device buffer pair with a head state (the reference's
    SyncedMemory, src/utils/blob.cc:83-143): each side is allocated lazily
    from the native pools; reading a side syncs it from the other when the
    other holds newer data; taking a side ``mutable_*`` makes it the only
    valid copy.  ``like=`` mirrors an existing device region (e.g. a
    parameter's slice of the flat store) instead of allocating one.

    Head states: 0 UNINITIALIZED, 1 HEAD_AT_CPU, 2 HEAD_AT_GPU, 3 SYNCED."""

    UNINITIALIZED, HEAD_AT_CPU, HEAD_AT_GPU, SYNCED = 0, 1, 2, 3

    def __init__(self, shape: Sequence[int], dtype=torch.float32, device=None, like: torch.Tensor = None,
                 pinned: bool = True):
        M = _mod()
        if M is None:
            raise RuntimeError("SyncedBlob needs the native library (_C)")
        self.shape = [int(s) for s in (like.shape if like is not None else shape)]
        self.dtype = like.dtype if like is not None else dtype
        code, bits = _CODES[self.dtype]
        self._cb = (code, bits)
        n = 1
        for s in self.shape:
            n *= s
        nbytes = n * bits // 8
        if like is not None:
            if not (like.is_cuda and like.is_contiguous()):
                raise ValueError("SyncedBlob(like=...) mirrors a dense device tensor")
            self.dev = like.device.index
            ext = like.data_ptr()
            self._keep = like
        else:
            d = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
            self.dev = d.index if d.index is not None else 0
            ext = 0
            self._keep = None
        self._b = M.SyncedBlob(max(nbytes, 1), self.dev, ext, pinned)
        self._M = M

    @property
    def head(self) -> int:
        return self._b.head

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream

    def _view(self, ptr: int, on_device: bool) -> torch.Tensor:
        code, bits = self._cb
        cap = self._M.blob_view(self._b, ptr, on_device, self.dev, _dl_device_type() if on_device else 1,
                                self.shape, code, bits)
        return torch.utils.dlpack.from_dlpack(cap)

    def cpu_data(self) -> torch.Tensor:
        return self._view(self._b.cpu_ptr(self._stream()), False)

    def gpu_data(self) -> torch.Tensor:
        return self._view(self._b.gpu_ptr(self._stream()), True)

    def mutable_cpu_data(self) -> torch.Tensor:
        return self._view(self._b.mutable_cpu_ptr(self._stream()), False)

    def mutable_gpu_data(self) -> torch.Tensor:
        return self._view(self._b.mutable_gpu_ptr(self._stream()), True)
