"""Loader and thin launch helpers for the gfx950 kernel library (``_C``).

The HIP path is the only GPU compute path for the ops implemented in
``singa_amd/csrc/kernels``: if the extension cannot be imported on a machine
with a GPU, :func:`lib` raises instead of silently falling back to PyTorch.
On CPU-only hosts the CPU reference implementations in
:mod:`singa_amd.ops.cpu` are used (they are the numerics oracle in tests).
"""
from __future__ import annotations

import importlib
import os

import torch

# dtype codes shared with csrc/kernels/common.h
F32, BF16, F16, I32, I64, U8 = 0, 1, 2, 3, 4, 5
_DT = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16, torch.int32: I32, torch.int64: I64,
       torch.uint8: U8}

_lib = None
_err = None


def _load():
    global _lib, _err
    if _lib is not None or _err is not None:
        return _lib
    try:
        _lib = importlib.import_module("singa_amd._C")
    except Exception as e:  # pragma: no cover - reported through lib()
        _err = e
        return _lib
    if os.environ.get("SINGA_AMD_DETERMINISTIC", "0") == "1" and hasattr(_lib, "set_deterministic"):
        _lib.set_deterministic(1)
    if os.environ.get("SINGA_BN_RPT") and hasattr(_lib, "bn_set_rows_per_thread"):
        _lib.bn_set_rows_per_thread(int(os.environ["SINGA_BN_RPT"]))  # 0: legacy grid-stride BN apply
    if os.environ.get("SINGA_AMD_CONV3X3", "1") == "0" and hasattr(_lib, "conv3x3_set"):
        _lib.conv3x3_set(0)  # persistent stage-1 3x3 conv off (A/B against the generic implicit GEMM)
    # kernel tuning knobs from the environment: SG_TUNE="0=4,1=1" (key=value)
    for kv in os.environ.get("SG_TUNE", "").split(","):
        if "=" in kv and hasattr(_lib, "set_tuning"):
            k, v = kv.split("=")
            _lib.set_tuning(int(k), int(v))
    # residual-tail GEMM knobs (bnres.hip sg_bnres_tune): SG_BNRES_TUNE="0=0"
    for kv in os.environ.get("SG_BNRES_TUNE", "").split(","):
        if "=" in kv and hasattr(_lib, "bnres_tune"):
            k, v = kv.split("=")
            _lib.bnres_tune(int(k), int(v))
    # fp32 generic-GEMM knobs (ggemm.hip sg_ggemm_tune): SG_GG_TUNE="2=1"
    for kv in os.environ.get("SG_GG_TUNE", "").split(","):
        if "=" in kv and hasattr(_lib, "ggemm_tune"):
            k, v = kv.split("=")
            _lib.ggemm_tune(int(k), int(v))
    return _lib


class _TracedLib:
    """SG_LAUNCH_TRACE=1: counts every binding call by (name, call site) --
    which Python lines launch the step's small kernels (tools/launch_sites.py)."""

    def __init__(self, m):
        import collections
        self._m = m
        self.counts = collections.Counter()
        self.enabled = False

    def __getattr__(self, k):
        v = getattr(self._m, k)
        if not callable(v) or not self.enabled or k in ("rt", "mem"):
            return v
        import sys

        f = sys._getframe(1)
        site = f"{f.f_code.co_filename.split('singa_amd/')[-1]}:{f.f_lineno}"
        f2 = f.f_back
        if f2 is not None:
            site += f" <- {f2.f_code.co_filename.split('singa_amd/')[-1]}:{f2.f_lineno}"

        def call(*a, **kw):
            self.counts[(k, site)] += 1
            return v(*a, **kw)
        return call


_TRACED = [None]


def lib():
    """Return the loaded ``_C`` module or raise a descriptive error."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "singa_amd native kernel library (_C) is not built or failed to load: "
            f"{_err!r}. Run `python -m singa_amd.build_ext`.")
    if os.environ.get("SG_LAUNCH_TRACE") == "1":
        if _TRACED[0] is None:
            _TRACED[0] = _TracedLib(m)
        return _TRACED[0]
    return m


def available() -> bool:
    return _load() is not None


def gpu_available() -> bool:
    return torch.cuda.is_available()


def dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype for native kernel: {t.dtype}")


_RAW = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_GETDEV = getattr(torch._C, "_cuda_getDevice", None)


_RT = [None]


def _rt():
    r = _RT[0]
    if r is None:
        lb = _load()
        r = _RT[0] = getattr(lb, "rt", None) if lb is not None else None
        if r is None:
            _RT[0] = False
    return r or None


def device() -> int:
    """This thread's current device (framework state: singa_amd.stream /
    device.py set it; the first query reads hipGetDevice)."""
    r = _rt()
    if r is not None:
        return r.get_device()
    return _GETDEV() if _GETDEV is not None else torch.cuda.current_device()


def stream(device: int | None = None) -> int:
    """Handle of this thread's current HIP stream: the framework stream this
    thread entered (singa_amd.stream.Stream), read from the native runtime
    -- no PyTorch call; when none is set, the caller's PyTorch current
    stream (the raw query: ~0.1 us)."""
    r = _rt()
    if r is not None:
        h = r.current(-1 if device is None else device)
        if h >= 0:
            return h
    if _RAW is not None and _GETDEV is not None:
        return _RAW(_GETDEV() if device is None else device)
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


def check(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


def is_cl(t: torch.Tensor) -> bool:
    """True if a 4-D tensor is dense channels_last (NHWC memory)."""
    return t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)


# Test-only hook: True routes GPU tensors to the PyTorch oracle expressions
# instead of the HIP kernels (a numerics experiment in a test).  There is no
# environment switch: the shipped op layer has exactly one device backend.
_TORCH_ORACLE_FOR_TESTS = [False]


def force_native() -> bool:
    """True: GPU tensors run on the HIP kernels (always, outside tests that
    flip the hook above)."""
    return not _TORCH_ORACLE_FOR_TESTS[0]
