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


_MOD = [None, False]


def _mod():
    if _MOD[1]:
        return _MOD[0]
    from .ops import native as N
    m = getattr(N.lib(), "mem", None) if N.available() else None
    _MOD[0], _MOD[1] = m, True
    return m


def _dl_device_type() -> int:
    """The DLPack device type this PyTorch build uses for GPU tensors (kDLROCM
    on ROCm builds), read from a tensor it exports."""
    global _DL_DEV
    if _DL_DEV is None:
        cap = torch.utils.dlpack.to_dlpack(torch.empty(1, device="cuda"))
        _DL_DEV = int(_mod().dl_device_type(cap))
    return _DL_DEV


_ON = [None]
_DEVS: dict = {None: torch.device("cpu"), "cpu": torch.device("cpu")}  # (pre-built: no torch.device call per allocation)
_RAWQ = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_GETD = getattr(torch._C, "_cuda_getDevice", None)


def _raw_stream(idx: int) -> int:
    from .ops import native as N
    return N.stream(idx)  # the framework's current stream (native state), else PyTorch's


def _getdev() -> int:
    from .ops import native as N
    return N.device()


def _native_on() -> bool:
    v = _ON[0]
    if v is None:
        v = _ON[0] = os.environ.get("SINGA_AMD_NATIVE_MEM", "1") != "0" and _mod() is not None
    return v


def enabled() -> bool:
    return _native_on()


def _cuda_index(dev) -> int:
    idx = dev.index
    return idx if idx is not None else torch.cuda.current_device()


def empty(*size, dtype=None, device=None, memory_format=None, pinned: bool = False, pin_memory: bool = False,
          **_ignored) -> torch.Tensor:
    """``torch.empty``'s signature; the storage is a block of a native pool:
    the device's HBM pool (stream-ordered on the current stream) or the
    64-byte-aligned / pinned host pool.  ``memory_format=torch.channels_last``
    lays a 4-D block out NHWC under the logical NCHW shape (one allocation,
    no copy).  ``SINGA_AMD_NATIVE_MEM=0`` (or no ``_C``): PyTorch's allocator."""
    if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)):
        size = size[0]
    elif len(size) >= 2 and isinstance(size[0], (tuple, list, torch.Size)):  # legacy empty(shape, dtype[, device])
        size, dtype, device = size[0], size[1], (size[2] if len(size) > 2 else device)
    dtype = dtype or torch.float32
    pinned = pinned or pin_memory
    dev = device if isinstance(device, torch.device) else _DEVS.get(device)
    if dev is None:
        dev = _DEVS[device] = torch.device(device if device is not None else "cpu")
    if not _native_on() or dtype not in _CODES:
        return torch.empty(tuple(size), dtype=dtype, device=dev, pin_memory=pinned and dev.type == "cpu",
                           memory_format=memory_format or torch.contiguous_format)
    M = _mod()
    shape = [int(v) for v in size]
    strides = []
    if memory_format is torch.channels_last and len(shape) == 4:
        n_, c_, h_, w_ = shape
        strides = [h_ * w_ * c_, 1, w_ * c_, c_]
    code, bits = _CODES[dtype]
    if dev.type == "cuda":
        idx = dev.index if dev.index is not None else _getdev()
        cap = M.empty(shape, code, bits, 0, idx, _DL_DEV or _dl_device_type(), _raw_stream(idx), strides)
    else:
        cap = M.empty(shape, code, bits, 2 if pinned else 1, 0, 1, 0, strides)
    t = torch.utils.dlpack.from_dlpack(cap)
    return t.view(torch.bool) if dtype == torch.bool and t.dtype != torch.bool else t


def empty_native(shape: Sequence[int], dtype=torch.float32, device=None, channels_last: bool = False,
                 pinned: bool = False):
    """A framework-owned tensor handle (``_C.mem.Tensor``: pool storage, byte
    offset, shape, strides, dtype, device -- csrc/mem/pool.cpp) over a new
    block of the device's HBM pool (stream-ordered on the current stream) or
    the host pool.  ``to_torch(h)`` / ``numpy.from_dlpack(h)`` view its bytes."""
    M = _mod()
    if M is None or not hasattr(M, "Tensor"):
        raise RuntimeError("the native tensor handle needs the _C extension")
    dev = device if isinstance(device, torch.device) else torch.device(device if device is not None else "cpu")
    code, bits = _CODES[dtype]
    shape = [int(v) for v in shape]
    if dev.type == "cuda":
        idx = dev.index if dev.index is not None else _getdev()
        return M.Tensor.empty(shape, code, bits, 0, idx, _DL_DEV or _dl_device_type(), _raw_stream(idx),
                              channels_last)
    return M.Tensor.empty(shape, code, bits, 2 if pinned else 1, 0, 1, 0, channels_last)


def native(t: torch.Tensor):
    """The native handle of any tensor's bytes (zero copy, DLPack: the handle
    keeps ``t``'s storage alive); views taken on it are native metadata."""
    M = _mod()
    if M is None or not hasattr(M, "Tensor"):
        raise RuntimeError("the native tensor handle needs the _C extension")
    return M.Tensor.from_dlpack(torch.utils.dlpack.to_dlpack(t))


def native_views() -> bool:
    """Tensor.reshape / transpose build their views on the native handle
    (``SINGA_AMD_NATIVE_VIEWS=0``: PyTorch's view machinery)."""
    v = _NV[0]
    if v is None:
        M = _mod()
        v = _NV[0] = (os.environ.get("SINGA_AMD_NATIVE_VIEWS", "1") != "0" and M is not None
                      and hasattr(M, "Tensor"))
    return v


_NV = [None]


def to_torch(h) -> torch.Tensor:
    """A torch view of a native handle's bytes (the view keeps the storage alive)."""
    t = torch.utils.dlpack.from_dlpack(h.to_dlpack())
    return t.view(torch.bool) if h.dtype == (6, 8) and t.dtype != torch.bool else t


def empty_like(t: torch.Tensor, dtype=None, memory_format=None) -> torch.Tensor:
    """Same shape (and, by default, the same dense layout: contiguous or
    channels_last) as ``t``."""
    if memory_format is None or memory_format is torch.preserve_format:
        memory_format = (torch.channels_last if t.dim() == 4 and not t.is_contiguous()
                         and t.is_contiguous(memory_format=torch.channels_last) else None)
    return empty(tuple(t.shape), dtype=dtype or t.dtype, device=t.device, memory_format=memory_format)


def record_stream(t: torch.Tensor, stream) -> None:
    """``t`` (or a view into a pool block) is used on ``stream`` too: its
    block is reused only after the work queued there so far completed
    (PyTorch's record_stream for tensors it allocated)."""
    if not t.is_cuda:
        return
    M = _mod()
    s = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
    if M is not None and _native_on() and M.owns(_cuda_index(t.device), t.data_ptr()):
        M.record_stream(_cuda_index(t.device), t.data_ptr(), s)
    else:
        ts = stream if isinstance(stream, torch.cuda.Stream) else (getattr(stream, "_ext", None) or
                                                                   torch.cuda.ExternalStream(s, device=t.device))
        t.record_stream(ts)  # a tensor PyTorch's allocator owns


class graph_pool:
    """Context manager: allocations of this thread go to a PRIVATE pool
    (a HIP graph's memory: blocks freed inside the capture are reused within
    it, and none of them is handed to work outside the graph).  ``release()``
    when the graph is destroyed."""

    def __init__(self, device=None):
        M = _mod()
        self.dev = _cuda_index(torch.device(device or "cuda"))
        self.id = M.new_pool(self.dev) if (M is not None and _native_on()) else 0
        self._prev = 0

    def __enter__(self):
        if self.id:
            self._prev = _mod().set_pool(self.id)
        return self

    def __exit__(self, *exc):
        if self.id:
            _mod().set_pool(self._prev)
        return False

    def release(self) -> None:
        if self.id:
            _mod().release_pool(self.dev, self.id)
            self.id = 0


def zeros(shape: Sequence[int], dtype=torch.float32, device="cpu") -> torch.Tensor:
    from .ops import glue as G
    return G.zero_(empty(tuple(shape), dtype=dtype, device=device))


def reset_peak(device=None) -> None:
    M = _mod()
    if M is not None:
        M.reset_peak(_cuda_index(torch.device(device or "cuda")))


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
