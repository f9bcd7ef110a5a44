"""Tracing / profiling.  The reference had only wall-clock
accumulators (``tForward_/tBackward_/tSyncData_``, src/worker/worker.cc:304-316)
and a per-layer norm1 debug dump; here:

* :func:`range` / :func:`mark` -- roctx ranges and markers (ROCm's
  ``libroctx64`` / rocprofiler-sdk roctx through ctypes), visible in
  ``rocprofv3 --marker-trace`` timelines next to the HIP kernels;
* :class:`ChromeTrace` -- an in-process event recorder that writes Chrome /
  Perfetto ``traceEvents`` JSON (HIP-event timed on a GPU, wall-clock on the
  CPU);
* :class:`LayerTracer` -- wraps every layer of a :class:`NeuralNet` (or a
  :class:`singa_amd.layer.Layer` tree) so each forward is a named range.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time
from typing import List, Optional

import torch

_ROCTX = {"lib": None, "tried": False}


def _roctx():
    if not _ROCTX["tried"]:
        _ROCTX["tried"] = True
        for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "libroctx64.so"):
            for d in ("/opt/rocm/lib", ""):
                try:
                    lib = ctypes.CDLL(os.path.join(d, name) if d else name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    _ROCTX["lib"] = lib
                    return lib
                except OSError:
                    continue
    return _ROCTX["lib"]


def enabled() -> bool:
    return os.environ.get("SINGA_AMD_ROCTX", "1") != "0" and _roctx() is not None


def push(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def pop() -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx/roctx naming
    push(name)
    try:
        yield
    finally:
        pop()


class ChromeTrace:
    """Collects (name, category, start, duration) events; GPU events are
    timed with HIP events and resolved lazily at :meth:`save`."""

    def __init__(self, gpu: Optional[bool] = None):
        self.gpu = torch.cuda.is_available() if gpu is None else gpu
        self.events: List = []
        self.t0 = time.perf_counter()
        self._lock = threading.Lock()
        if self.gpu:
            from .. import stream as _stream
            self._Ev = _stream.Event
            self.e0 = _stream.Event(timing=True)
            self.e0.record()

    @contextlib.contextmanager
    def span(self, name: str, cat: str = "layer", args: Optional[dict] = None):
        push(name)
        if self.gpu:
            a, b = self._Ev(timing=True), self._Ev(timing=True)
            a.record()
            try:
                yield
            finally:
                b.record()
                pop()
                with self._lock:
                    self.events.append((name, cat, a, b, args))
        else:
            s = time.perf_counter()
            try:
                yield
            finally:
                e = time.perf_counter()
                pop()
                with self._lock:
                    self.events.append((name, cat, (s - self.t0) * 1e3, (e - s) * 1e3, args))

    def to_json(self, pid: int = 0) -> dict:
        if self.gpu:
            torch.cuda.synchronize()
        ev = []
        for name, cat, a, b, args in self.events:
            if self.gpu:
                ts, dur = self.e0.elapsed_time(a), a.elapsed_time(b)
            else:
                ts, dur = a, b
            e = {"name": name, "cat": cat, "ph": "X", "ts": ts * 1e3, "dur": dur * 1e3, "pid": pid, "tid": 0}
            if args:
                e["args"] = args
            ev.append(e)
        return {"traceEvents": ev, "displayTimeUnit": "ms"}

    def save(self, path: str, pid: int = 0) -> None:
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(self.to_json(pid), f)

    def summary(self) -> dict:
        """name -> (calls, total ms)."""
        out = {}
        for e in self.to_json()["traceEvents"]:
            c, t = out.get(e["name"], (0, 0.0))
            out[e["name"]] = (c + 1, t + e["dur"] / 1e3)
        return out


class LayerTracer:
    """Instrument every layer's ``forward`` of a config-path NeuralNet (or
    the sub-layers of a python-API Model) with a trace span."""

    def __init__(self, net, dev=None, trace: Optional[ChromeTrace] = None):
        gpu = dev is not None and getattr(dev, "torch_device", torch.device("cpu")).type == "cuda"
        self.trace = trace or ChromeTrace(gpu=gpu)
        self._wrapped = []
        layers = getattr(net, "layers", None)
        if layers is None:  # python-API Model: walk sub-layers
            layers = [l for _, l in _walk(net)]
        for l in layers:
            self._wrap(l)

    def _wrap(self, l):
        orig = l.forward
        name = getattr(l, "name", type(l).__name__)
        tr = self.trace

        def fwd(*a, **k):
            with tr.span(str(name), "forward"):
                return orig(*a, **k)

        l.forward = fwd
        self._wrapped.append((l, orig))

    def remove(self):
        for l, orig in self._wrapped:
            l.forward = orig
        self._wrapped.clear()

    def save(self, path: str, pid: int = 0):
        self.trace.save(path, pid)


def _walk(m, prefix=""):
    for k, v in vars(m).items():
        from ..layer import Layer

        if isinstance(v, Layer):
            name = f"{prefix}{k}"
            v.name = getattr(v, "name", None) or name
            yield name, v
            yield from _walk(v, name + ".")
