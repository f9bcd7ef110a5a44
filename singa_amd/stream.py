"""Framework-owned HIP streams, events and step graphs (``_C.rt``,
csrc/mem/stream_graph.cpp).

* :class:`Stream` -- a native non-blocking stream (priority selectable).
  ``with s:`` makes it the current stream of this thread for every launcher
  (PyTorch's current-stream slot is only the carrier: the handle is wrapped
  as an ``ExternalStream``, nothing is created by PyTorch).
* :class:`Event` -- record / wait (device-side join) / query / synchronize /
  elapsed_ms.
* :class:`StepGraph` -- capture of a training step on a framework stream with
  ``hipStreamBeginCapture`` (thread-local mode), one instantiation, replay
  with ``hipGraphLaunch``; the step's memory comes from a private native pool
  (:class:`singa_amd.memory.graph_pool`) that lives exactly as long as the
  graph.  This is :class:`singa_amd.model.Model`'s graph executor.

Reference: the reference had no device-side execution machinery (its CUDA
path, include/mshadow/tensor_gpu-inl.hpp:26-93, was compiled out); its
overlap came from ZeroMQ actor threads (src/server/server.cc:53-60).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from .ops import native as N


def _rt():
    return N.lib().rt


def device_synchronize(device=None) -> None:
    """Wait until every stream of ``device`` is idle (hipDeviceSynchronize)."""
    idx = torch.device(device).index if isinstance(device, (str, torch.device)) else device
    _rt().device_synchronize(-1 if idx is None else int(idx))


def current(device=None) -> int:
    """Handle of this thread's current stream on ``device``."""
    idx = torch.device(device).index if isinstance(device, (str, torch.device)) else device
    return N.stream(idx)


def is_capturing(stream=None) -> bool:
    """True while ``stream`` (default: this thread's current stream) is being
    captured into a HIP graph (hipStreamIsCapturing)."""
    return bool(_rt().is_capturing(_handle(stream)))


class Stream:
    def __init__(self, device=None, priority: int = 0):
        idx = torch.device(device).index if device is not None else None
        self.device_index = idx if idx is not None else N.device()
        self._s = _rt().Stream(self.device_index, int(priority))
        self.handle = self._s.handle
        # the carrier through which ``with stream:`` sets the current stream
        self._ext = torch.cuda.ExternalStream(self.handle, device=torch.device("cuda", self.device_index))
        self._ctx = __import__("threading").local()  # per-thread stack: threads may enter one stream together

    @property
    def cuda_stream(self) -> int:  # duck-typing with torch.cuda.Stream for launch helpers
        return self.handle

    def wait_stream(self, other) -> None:
        """This stream waits (device-side) for the work queued so far on ``other``."""
        if _handle(other) == self.handle:
            return  # stream order already
        ev = Event()
        ev.record(other)
        ev.wait(self)

    def synchronize(self) -> None:
        self._s.synchronize()

    def query(self) -> bool:
        return self._s.query()

    def __enter__(self):
        # the framework's own current stream (read by every launcher, no
        # PyTorch query), and PyTorch's slot too, for torch ops in tests
        old = _rt().set_current(self.device_index, self.handle)
        ctx = torch.cuda.stream(self._ext)
        ctx.__enter__()
        st = getattr(self._ctx, "stack", None)
        if st is None:
            st = self._ctx.stack = []
        st.append((ctx, old))
        return self

    def __exit__(self, *exc):
        ctx, old = self._ctx.stack.pop()
        _rt().set_current(self.device_index, old)
        return ctx.__exit__(*exc)


_POOLED: dict = {}


def pooled(device=None, role: str = "side", priority: int = 0) -> Stream:
    """The framework stream of ``role`` on ``device`` (created once, reused):
    the native pool caches freed blocks per stream, so a stream created per
    call (and never destroyed) would strand its cached blocks; prefetchers,
    communicators, executor threads and rank threads take theirs from here."""
    idx = torch.device(device).index if device is not None else None
    idx = idx if idx is not None else torch.cuda.current_device()
    key = (idx, role, int(priority))
    s = _POOLED.get(key)
    if s is None:
        s = _POOLED[key] = Stream(torch.device("cuda", idx), priority=priority)
    return s


def _handle(s) -> int:
    if s is None:
        return current()
    if isinstance(s, int):
        return s
    return s.cuda_stream


class Event:
    def __init__(self, timing: bool = False):
        self._e = _rt().Event(bool(timing))

    def record(self, stream=None) -> "Event":
        self._e.record(_handle(stream))
        return self

    def wait(self, stream=None) -> None:
        """``stream`` (default: current) waits on the device for this event."""
        self._e.wait(_handle(stream))

    def query(self) -> bool:
        return self._e.query()

    def synchronize(self) -> None:
        self._e.synchronize()

    def elapsed_time(self, end: "Event") -> float:
        return self._e.elapsed_ms(end._e)


_CAPTURE_STREAMS: dict = {}
_TLS = __import__("threading").local()


def set_step_graph_factory(factory) -> None:
    """This thread's models capture their steps with ``factory(device)``
    instead of :class:`StepGraph` (None restores the default).  The loopback
    world's rank threads install their rank's :class:`~singa_amd.parallel.loop.WorldGraph`
    view here, so every rank's step lands in ONE graph."""
    _TLS.factory = factory


def new_step_graph(device=None):
    f = getattr(_TLS, "factory", None)
    return f(device) if f is not None else StepGraph(device)


class StepGraph:
    """One captured step: ``capture(fn, *args)`` runs fn once under capture
    (nothing executes) on a framework stream forked from the current one and
    returns fn's result -- the graph's static outputs; ``replay()`` launches
    the instantiated graph on the current stream."""

    def __init__(self, device=None):
        from . import memory

        idx = torch.device(device).index if device is not None else None
        self.device_index = idx if idx is not None else torch.cuda.current_device()
        self._g = _rt().Graph()
        self.pool = memory.graph_pool(torch.device("cuda", self.device_index))
        self.keep: list = []
        self._arena = 0  # the persistent kernels' queue slots of this graph (workq.hip)

    def capture(self, fn: Callable, *args, **kwargs):
        s = _CAPTURE_STREAMS.get(self.device_index)
        if s is None:
            s = _CAPTURE_STREAMS[self.device_index] = Stream(torch.device("cuda", self.device_index))
        cur = current(self.device_index)
        s.wait_stream(cur)
        torch_before = torch.cuda.memory_allocated(self.device_index)
        L = N.lib()
        with s, self.pool:
            self._arena = L.workq_arena_begin()
            try:
                self._g.begin(s.handle)
                try:
                    out = fn(*args, **kwargs)
                except BaseException:
                    self._g.abort()
                    raise
                self._g.end()
            finally:
                L.workq_arena_end()
        if torch.cuda.memory_allocated(self.device_index) != torch_before:
            # a PyTorch allocation inside the capture would live in PyTorch's
            # allocator, which does not know the graph still uses it
            raise RuntimeError("StepGraph: the captured step allocated through PyTorch's allocator")
        Event().record(s).wait(cur)
        return out

    @property
    def nodes(self) -> int:
        return self._g.nodes

    def replay(self) -> None:
        self._g.replay(current(self.device_index))

    @property
    def queue_slots(self) -> int:
        """Work-queue slots the captured persistent kernels hold."""
        return N.lib().workq_arena_slots(self._arena) if self._arena else 0

    def release(self) -> None:
        self._g.reset()
        self.pool.release()
        if self._arena:
            N.lib().workq_arena_free(self._arena)
            self._arena = 0
