"""Loopback ranks: run N ranks as N threads of this process over the native
RCCL call surface (``_C.LoopComm``, csrc/comm/loop_comm.cpp), each wrapped in
the real :class:`~singa_amd.parallel.rccl.RcclCommunicator`.

This is how the multi-rank RCCL path -- the wrapper's async fork / join on a
comm stream, DistOpt's fp32 / bf16 bucket exchange, the sharded EASGD centre,
the grouped point-to-point pipeline bridges -- runs at world sizes 2..8 on ONE
GPU (``device=torch.device("cuda", 0)``: each rank thread gets its own compute
stream) or on host memory in CPU CI (``device=None``).  The exchange itself is
synchronous host staging, so it proves correctness of everything above the
transport, not xGMI bandwidth.  (The reference exercised its exchange only as
real multi-process ZeroMQ traffic: src/utils/param_manager.cc:103-234.)

``run_ranks(..., captured=True)`` runs the ranks' HIP-graph steps as ONE
graph (:class:`WorldGraph`): each rank thread's ``Model(use_graph=True)``
capture joins a capture rooted on a world stream, the bucket all-reduces that
DistOpt forks onto each rank's comm stream inside the captured backward
become graph edges plus a device reduction (LoopComm's captured mode), and a
replay launches every rank's step at once.  That is the N > 1 timed path of
``bench.py`` -- collectives inside the captured step -- executed with N ranks
on one GPU.
"""
from __future__ import annotations

import os
import sys
import threading
from typing import Callable, List, Optional

import torch

from .. import stream as _stream
from ..ops import native as N
from .rccl import RcclCommunicator


_DBG = os.environ.get("SG_LOOP_DEBUG") == "1"


def _dbg(*a) -> None:
    if _DBG:
        print(f"[{threading.current_thread().name}]", *a, file=sys.stderr, flush=True)


class WorldGraph:
    """One HIP graph holding the captured steps of every rank thread of a
    loopback world on one GPU.

    Each rank thread's models get a :meth:`view` (through
    :func:`singa_amd.stream.set_step_graph_factory`) with StepGraph's
    ``capture`` / ``replay`` / ``release``.  ``capture``: all ranks meet,
    rank 0 begins a capture on the world's origin stream, and every rank runs
    its step body with the ORIGIN as its current stream and its
    communicator's comm stream (its own private memory pool and work-queue
    arena): stream order then carries every dependency, and a collective is
    one device reduction enqueued once all ranks have reached it (LoopComm's
    captured mode).  Rank 0 ends the capture.  ``replay``: all ranks meet
    (each one's ``prepare_step`` kernels fenced in with an event), rank 0
    launches the graph on the origin stream, and every rank's stream waits for
    it.  A rank that fails breaks the barrier, so its peers fail instead of
    waiting.

    The ranks' work is serialised on one stream inside the graph: this checks
    the captured step's logic at N ranks (buckets reduced inside the graph,
    replicas in lock-step), not cross-rank concurrency.  Side streams that
    wait on each other's events from two rank threads were the first design;
    this HIP runtime's hipStreamEndCapture crashes on such a capture
    (tools/capture_threads_probe.py xrank1)."""

    def __init__(self, world: int, device: torch.device, timeout_s: float = 120.0):
        self.world = world
        self.device = torch.device(device)
        self.dev = self.device.index or 0
        self.timeout_s = timeout_s
        self.bar = threading.Barrier(world)
        self.origin = _stream.Stream(self.device)
        self._g = N.lib().rt.Graph()
        self.comms: List[object] = [None] * world  # each rank's communicator (its comm stream swapped during capture)
        self.events: List[object] = [None] * world
        self.done = None
        self.captures = 0
        self.replays = 0

    def _meet(self) -> None:
        self.bar.wait(self.timeout_s)

    def abort(self) -> None:
        self.bar.abort()

    def view(self, rank: int):
        return _RankGraph(self, rank)

    @property
    def nodes(self) -> int:
        return self._g.nodes


class _RankGraph:
    """Rank ``rank``'s handle on a :class:`WorldGraph` (StepGraph interface)."""

    def __init__(self, wg: WorldGraph, rank: int):
        from .. import memory

        self.wg, self.rank = wg, rank
        self.pool = memory.graph_pool(wg.device)
        self._arena = 0

    def capture(self, fn: Callable, *args, **kwargs):
        wg, L = self.wg, N.lib()
        began = False
        try:
            wg._meet()
            if self.rank == 0:
                _dbg("begin capture")
                wg._g.begin(wg.origin.handle, 2)  # relaxed: every rank thread enqueues into this capture
                began = True
            wg._meet()
            comm = wg.comms[self.rank]
            saved = getattr(comm, "comm_stream", None)
            if comm is not None:
                comm.comm_stream = wg.origin
            try:
                with wg.origin, self.pool:
                    self._arena = L.workq_arena_begin()
                    try:
                        _dbg("body")
                        out = fn(*args, **kwargs)
                    finally:
                        L.workq_arena_end()
            finally:
                if comm is not None:
                    comm.comm_stream = saved
            _dbg("body done")
            wg._meet()
            if self.rank == 0:
                _dbg("end capture")
                wg._g.end()
                _dbg("instantiated", wg._g.nodes)
                began = False
                wg.captures += 1
            wg._meet()
            return out
        except BaseException:
            wg.abort()
            if began:
                wg._g.abort()
            raise

    @property
    def nodes(self) -> int:
        return self.wg.nodes

    def replay(self) -> None:
        wg = self.wg
        cur = _stream.current(wg.dev)
        wg.events[self.rank] = _stream.Event().record(cur)  # this rank's prepare_step work
        wg._meet()
        if self.rank == 0:
            try:
                for ev in wg.events:
                    ev.wait(wg.origin)
                _dbg("replay")
                wg._g.replay(wg.origin.handle)
                wg.done = _stream.Event().record(wg.origin)
                wg.replays += 1
            except BaseException:
                wg.abort()
                raise
        wg._meet()
        wg.done.wait(cur)

    def release(self) -> None:
        wg = self.wg
        try:
            wg._meet()
        except threading.BrokenBarrierError:
            pass
        if self.rank == 0:
            wg._g.reset()
        try:
            wg._meet()
        except threading.BrokenBarrierError:
            pass
        self.pool.release()
        if self._arena:
            N.lib().workq_arena_free(self._arena)
            self._arena = 0


def run_ranks(fn: Callable, world: int, *args, device: Optional[torch.device] = None, timeout_s: float = 60.0,
              return_exceptions: bool = False, captured: bool = False) -> List[object]:
    """Run ``fn(rank, world, comm, *args)`` on ``world`` threads sharing one
    loopback world; returns the per-rank results in rank order (re-raising
    the first failure unless ``return_exceptions``).  A failing rank aborts
    the world, so its peers fail fast instead of waiting for the timeout.
    ``captured=True`` (device ranks): the ranks' HIP-graph steps are captured
    into one :class:`WorldGraph` (``fn`` may read it as ``comm.world_graph``)."""
    L = N.lib()
    lw = L.LoopWorld(world, float(timeout_s))
    dev = -1 if device is None or torch.device(device).type == "cpu" else (torch.device(device).index or 0)
    if captured and dev < 0:
        raise ValueError("run_ranks(captured=True) needs device ranks")
    wg = WorldGraph(world, torch.device("cuda", dev), timeout_s) if captured else None
    res: List[object] = [None] * world
    errs: List[Optional[BaseException]] = [None] * world

    def body(r: int) -> None:
        native = L.LoopComm(lw, r, dev)
        try:
            if dev >= 0:
                torch.cuda.set_device(dev)
                s = _stream.pooled(torch.device("cuda", dev), f"loop-rank{r}")
                if wg is not None:
                    _stream.set_step_graph_factory(lambda device, r=r: wg.view(r))
                try:
                    with s:
                        comm = RcclCommunicator(world, r, r, native=native, device=torch.device("cuda", dev))
                        comm.world_graph = wg
                        if wg is not None:
                            wg.comms[r] = comm
                        res[r] = fn(r, world, comm, *args)
                    s.synchronize()
                finally:
                    _stream.set_step_graph_factory(None)
            else:
                comm = RcclCommunicator(world, r, r, native=native)
                res[r] = fn(r, world, comm, *args)
        except BaseException as e:  # noqa: BLE001 - reported to the caller
            errs[r] = e
            native.abort()
            if wg is not None:
                wg.abort()

    ts = [threading.Thread(target=body, args=(r,), daemon=True, name=f"loop-rank-{r}") for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout_s * 4)
    if any(t.is_alive() for t in ts):
        raise TimeoutError("loopback ranks did not finish")
    if return_exceptions:
        return [errs[r] if errs[r] is not None else res[r] for r in range(world)]
    first = next((e for e in errs if e is not None and "aborted" not in str(e)), None)
    first = first or next((e for e in errs if e is not None), None)
    if first is not None:
        raise first
    return res
