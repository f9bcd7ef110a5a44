"""Devices: ``CppCPU`` (native C++ host kernels, csrc/runtime/cpu_ops.cc) and ``RocmGPU``.

Mirrors the SINGA python device API (``create_cuda_gpu``, ``get_default_device``,
``Device.SetRandSeed``, ``EnableGraph``, ``Sync``, ``PrintTimeProfiling`` ...)
with one GPU class -- there is no CUDA/OpenCL dual path.  The reference's
devices are mshadow's compile-time ``cpu``/``gpu`` tags
(include/mshadow/tensor.h:185-200) with the GPU backend compiled out
(Makefile:17-19); here a device owns a torch device (HIP caching allocator),
a counter-based RNG stream (seed, offset) for the Philox kernels, a graph
flag used by :class:`singa_amd.model.Model`, and per-op HIP-event timers.
"""
from __future__ import annotations

import os
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch


class Device:
    lang_name = "base"

    def __init__(self, torch_device: torch.device, dev_id: int = -1):
        self.torch_device = torch.device(torch_device)
        self._id = dev_id
        self.seed = 0
        self.rng_offset = 0
        self.graph_enabled = False
        self.verbosity = 0
        self.skip_iteration = 5
        self._timings: Dict[str, List[float]] = defaultdict(list)
        self.generator = torch.Generator(device=self.torch_device)
        self.generator.manual_seed(0)

    # --- SINGA device API -------------------------------------------------
    def id(self) -> int:
        return self._id

    def lang(self) -> str:
        return self.lang_name

    def SetRandSeed(self, seed: int) -> None:
        self.seed = int(seed)
        self.rng_offset = 0
        self.generator.manual_seed(int(seed))

    def next_rng(self, n: int) -> tuple:
        """Reserve n Philox counters; returns (seed, offset)."""
        off = self.rng_offset
        self.rng_offset += (int(n) + 3) // 4
        return self.seed, off

    def rng_epoch(self) -> Optional[torch.Tensor]:
        """Device-resident int64 step counter for graph-safe RNG (GPU only):
        RNG kernels mix it into their Philox key; a captured training step
        advances it (:meth:`advance_rng_epoch`), so every replay differs."""
        if self.torch_device.type != "cuda":
            return None
        if getattr(self, "_rng_epoch", None) is None:
            from .ops import glue as G
            self._rng_epoch = G.zeros((1,), torch.int64, self.torch_device)
        return self._rng_epoch

    def advance_rng_epoch(self) -> None:
        ep = self.rng_epoch()
        if ep is not None:
            from .ops import glue as G
            G.iadd_(ep, 1)

    def EnableGraph(self, enable: bool) -> None:
        self.graph_enabled = bool(enable)

    def graph_enabled_(self) -> bool:
        return self.graph_enabled

    def Sync(self) -> None:
        if self.torch_device.type == "cuda":
            torch.cuda.synchronize(self.torch_device)

    def ResetGraph(self) -> None:
        pass

    def SetVerbosity(self, v: int) -> None:
        self.verbosity = int(v)

    def SetSkipIteration(self, n: int) -> None:
        self.skip_iteration = int(n)

    def record_time(self, name: str, ms: float) -> None:
        self._timings[name].append(ms)

    def PrintTimeProfiling(self) -> str:
        lines = []
        for k, v in self._timings.items():
            vv = v[self.skip_iteration:] or v
            lines.append(f"{k}: {sum(vv) / len(vv):.3f} ms (n={len(vv)})")
        s = "\n".join(lines)
        print(s)
        return s

    def is_gpu(self) -> bool:
        return self.torch_device.type == "cuda"

    def __repr__(self):
        return f"{type(self).__name__}(id={self._id})"

    def __eq__(self, other):
        return isinstance(other, Device) and self.torch_device == other.torch_device

    def __hash__(self):
        return hash(str(self.torch_device))


class CppCPU(Device):
    """Host device: its tensors' compute runs on the native C++ kernels of
    ``_core.cpu`` (threaded packed GEMM, im2col convolution, pooling, LRN,
    softmax-xent, normalisation, elementwise / broadcast / reduction loops;
    see :mod:`singa_amd.ops.cpu`).  PyTorch supplies host storage only."""
    lang_name = "kCpp"

    def __init__(self):
        super().__init__(torch.device("cpu"), -1)


class RocmGPU(Device):
    """One MI355X (gfx950) device.  All hot ops run hand-written HIP kernels."""
    lang_name = "kHip"

    def __init__(self, dev_id: int = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("RocmGPU requested but no HIP device is visible")
        super().__init__(torch.device("cuda", dev_id), dev_id)
        from .ops import native

        native.lib()  # fail loudly if the kernel library is missing

    def properties(self) -> dict:
        p = torch.cuda.get_device_properties(self.torch_device)
        return {"name": p.name, "gcnArchName": getattr(p, "gcnArchName", ""), "total_memory": p.total_memory,
                "multi_processor_count": p.multi_processor_count}


_default_cpu: Optional[CppCPU] = None
_gpus: Dict[int, RocmGPU] = {}
_default: Optional[Device] = None


def get_default_device() -> Device:
    global _default, _default_cpu
    if _default is None:
        if _default_cpu is None:
            _default_cpu = CppCPU()
        _default = _default_cpu
    return _default


def set_default_device(dev: Device) -> None:
    global _default
    _default = dev


def create_cpu_device() -> CppCPU:
    global _default_cpu
    if _default_cpu is None:
        _default_cpu = CppCPU()
    return _default_cpu


def get_num_gpus() -> int:
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def get_gpu_ids() -> List[int]:
    return list(range(get_num_gpus()))


def create_rocm_gpu_on(device_id: int, set_default: bool = False) -> RocmGPU:
    if device_id not in _gpus:
        _gpus[device_id] = RocmGPU(device_id)
    d = _gpus[device_id]
    if set_default:
        set_default_device(d)
    return d


def create_rocm_gpu(set_default: bool = False) -> RocmGPU:
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = max(get_num_gpus(), 1)
    return create_rocm_gpu_on(local % n, set_default)


def create_rocm_gpus(num: int) -> List[RocmGPU]:
    return [create_rocm_gpu_on(i) for i in range(num)]


def create_rocm_gpus_on(device_ids: List[int]) -> List[RocmGPU]:
    return [create_rocm_gpu_on(i) for i in device_ids]


# SINGA-compatible aliases (user code written for singa.device keeps working)
create_cuda_gpu = create_rocm_gpu
create_cuda_gpu_on = create_rocm_gpu_on
create_cuda_gpus = create_rocm_gpus
create_cuda_gpus_on = create_rocm_gpus_on


def best_device() -> Device:
    """RocmGPU when a GPU is visible, else CppCPU."""
    return create_rocm_gpu() if get_num_gpus() > 0 else create_cpu_device()


class Timer:
    """Wall-clock / HIP-event timer reproducing the reference's TimerInfo
    fwd/bwd/sync split (include/worker/worker.h:91-114)."""

    def __init__(self, dev: Device):
        self.dev = dev
        self.gpu = dev.is_gpu()

    def __enter__(self):
        if self.gpu:
            from . import stream as _stream
            self.s = _stream.Event(timing=True)
            self.e = _stream.Event(timing=True)
            self.s.record()
        else:
            self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        if self.gpu:
            self.e.record()
            self.e.synchronize()
            self.ms = self.s.elapsed_time(self.e)
        else:
            self.ms = (time.perf_counter() - self.t0) * 1e3
        return False
