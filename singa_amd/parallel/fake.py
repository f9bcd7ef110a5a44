"""In-process fake communicator: N ranks as N threads over shared host memory,
with fault injection (SURVEY §4 item 3, §5.3, §5.8 "Fake backend").

The reference tested distribution only with real processes over TCP
(examples/mnist/run.sh, src/test/test_pm.cc) and had no way to make a rank
fail on purpose; its only failure handling was the 10 x 1 s PING retry in
``Router::Connect`` (src/utils/router.cc:21-43).  This module lets CPU CI
exercise every caller of :class:`~singa_amd.parallel.Communicator` (DistOpt,
EASGD / RandomSync, bridges, the Worker) deterministically and cheaply, and
inject the failures the RCCL path must survive:

* ``FaultPlan.delay(rank, op, seconds)``  -- a straggler (results unchanged);
* ``FaultPlan.drop(rank, op, nth)``       -- a lost message: the peers of that
  collective / the receiver of that send time out with :class:`CommTimeout`;
* ``FaultPlan.kill(rank, op, nth)``       -- the rank raises :class:`RankKilled`
  at its ``nth`` call of ``op``; every peer blocked on it gets
  :class:`CommTimeout` after ``timeout_s`` (the watchdog of §5.3).

Collective semantics are those of RCCL: every rank calls the same sequence of
collectives on a group; ``all_reduce`` etc. work in place on ``torch.Tensor``s.
``run_threads(fn, world)`` spawns the ranks and returns per-rank results (or
re-raises the first failure).
"""
from __future__ import annotations

import queue
import threading
import time
from collections import defaultdict
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch


class CommTimeout(RuntimeError):
    """A collective / receive did not complete within the watchdog timeout."""


class RankKilled(RuntimeError):
    """Raised inside a rank that a :class:`FaultPlan` killed."""


class FaultPlan:
    """Per-(rank, op) fault schedule.  ``op`` names a Communicator method
    ("all_reduce", "broadcast", "send", ...) or "*" for any of them; ``nth``
    counts that rank's calls of ``op`` from 1."""

    def __init__(self):
        self._delays: Dict[Tuple[int, str], float] = {}
        self._drops: Dict[Tuple[int, str], set] = defaultdict(set)
        self._kills: Dict[Tuple[int, str], int] = {}
        self._counts: Dict[Tuple[int, str], int] = defaultdict(int)
        self._lock = threading.Lock()
        self.log: List[tuple] = []

    def delay(self, rank: int, op: str = "*", seconds: float = 0.05) -> "FaultPlan":
        self._delays[(rank, op)] = seconds
        return self

    def drop(self, rank: int, op: str = "*", nth: int = 1) -> "FaultPlan":
        self._drops[(rank, op)].add(nth)
        return self

    def kill(self, rank: int, op: str = "*", nth: int = 1) -> "FaultPlan":
        self._kills[(rank, op)] = nth
        return self

    def on_call(self, rank: int, op: str) -> bool:
        """Apply the plan to one call; returns False when the call's
        contribution must be dropped."""
        with self._lock:
            n_op = self._counts[(rank, op)] = self._counts[(rank, op)] + 1
            n_any = self._counts[(rank, "*")] = self._counts[(rank, "*")] + 1
        for key, n in (((rank, op), n_op), ((rank, "*"), n_any)):
            if self._kills.get(key) == n:
                self.log.append(("kill", rank, op, n))
                raise RankKilled(f"rank {rank} killed at call {n} of {key[1]}")
        d = self._delays.get((rank, op), self._delays.get((rank, "*"), 0.0))
        if d:
            self.log.append(("delay", rank, op, d))
            time.sleep(d)
        for key, n in (((rank, op), n_op), ((rank, "*"), n_any)):
            if n in self._drops.get(key, ()):
                self.log.append(("drop", rank, op, n))
                return False
        return True


class _Done:
    """Completed async handle (the fake backend finishes work eagerly)."""

    def wait(self, timeout=None):
        return True

    def is_completed(self):
        return True


class _Group:
    """Rendezvous state shared by the ranks of one (sub-)group."""

    def __init__(self, ranks: Sequence[int], timeout_s: float):
        self.ranks = list(ranks)
        self.n = len(self.ranks)
        self.timeout_s = timeout_s
        self.cv = threading.Condition()
        self.seq = [0] * self.n           # per-rank collective sequence number
        self.slots: Dict[int, dict] = defaultdict(dict)  # seq -> {rank: payload}
        self.done: Dict[int, int] = defaultdict(int)      # seq -> ranks finished reading
        self.dropped: Dict[int, bool] = {}

    def exchange(self, r: int, payload, keep: bool) -> List:
        """Deposit ``payload`` for this rank's next collective and return every
        rank's payload (in group order) once all have arrived."""
        with self.cv:
            s = self.seq[r]
            self.seq[r] += 1
            if keep:
                self.slots[s][r] = payload
            else:
                self.dropped[s] = True
            self.cv.notify_all()
            t_end = time.monotonic() + self.timeout_s
            while len(self.slots[s]) < self.n:
                if self.dropped.get(s) and len(self.slots[s]) + 1 >= self.n:
                    break
                left = t_end - time.monotonic()
                if left <= 0:
                    raise CommTimeout(f"collective #{s} timed out after {self.timeout_s}s on rank {r} "
                                      f"({len(self.slots[s])}/{self.n} ranks arrived)")
                self.cv.wait(left)
            if self.dropped.get(s):
                raise CommTimeout(f"collective #{s}: a contribution was lost (rank {r} sees "
                                  f"{len(self.slots[s])}/{self.n})")
            out = [self.slots[s][i] for i in range(self.n)]
            self.done[s] += 1
            if self.done[s] == self.n:
                del self.slots[s], self.done[s]
            return out


class FakeWorld:
    """Shared state of one fake job: the world group, sub-groups (created on
    first ``split``) and point-to-point mailboxes."""

    def __init__(self, world_size: int, timeout_s: float = 10.0, faults: Optional[FaultPlan] = None):
        self.world_size = world_size
        self.timeout_s = timeout_s
        self.faults = faults or FaultPlan()
        self.world = _Group(range(world_size), timeout_s)
        self._groups: Dict[tuple, _Group] = {}
        self._lock = threading.Lock()
        self._boxes: Dict[tuple, queue.Queue] = defaultdict(queue.Queue)

    def group(self, ranks: Sequence[int]) -> _Group:
        key = tuple(ranks)
        with self._lock:
            g = self._groups.get(key)
            if g is None:
                g = self._groups[key] = _Group(key, self.timeout_s)
            return g

    def box(self, src: int, dst: int) -> queue.Queue:
        with self._lock:
            return self._boxes[(src, dst)]

    def communicator(self, rank: int) -> "FakeCommunicator":
        return FakeCommunicator(self, self.world, rank)


class FakeCommunicator:
    """Drop-in for :class:`singa_amd.parallel.Communicator` (same method
    names and in-place tensor semantics)."""

    backend = "fake"

    def __init__(self, world: FakeWorld, group: _Group, rank: int, global_rank: Optional[int] = None):
        self.fw = world
        self.g = group
        self.world_size = group.n
        self.rank = rank
        self.global_rank = group.ranks[rank] if global_rank is None else global_rank
        self.local_rank = self.global_rank
        self.ranks = list(group.ranks)

    # ------------------------------------------------------------- helpers
    def _enter(self, op: str) -> bool:
        return self.fw.faults.on_call(self.global_rank, op)

    def _xchg(self, op: str, payload) -> List:
        keep = self._enter(op)
        return self.g.exchange(self.rank, payload, keep)

    @staticmethod
    def _ret(async_op: bool):
        return _Done() if async_op else None

    # --------------------------------------------------------- collectives
    def split(self, ranks: List[int]) -> Optional["FakeCommunicator"]:
        ranks = sorted(int(r) for r in ranks)
        self._xchg("split", None)  # collective, like dist.new_group
        if self.global_rank not in ranks:
            return None
        return FakeCommunicator(self.fw, self.fw.group(ranks), ranks.index(self.global_rank), self.global_rank)

    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = False):
        if self.world_size == 1:
            return self._ret(async_op)
        parts = self._xchg("all_reduce", t.detach().clone())
        acc = parts[0].clone()
        for p in parts[1:]:
            if op in ("sum", "avg"):
                acc.add_(p)
            elif op == "max":
                torch.maximum(acc, p, out=acc)
            elif op == "min":
                torch.minimum(acc, p, out=acc)
            else:
                raise ValueError(op)
        if op == "avg":
            acc.div_(self.world_size)
        t.copy_(acc)
        return self._ret(async_op)

    def broadcast(self, t: torch.Tensor, src: int = 0, async_op: bool = False):
        if self.world_size == 1:
            return self._ret(async_op)
        parts = self._xchg("broadcast", t.detach().clone() if self.rank == src else None)
        if self.rank != src:
            t.copy_(parts[src])
        return self._ret(async_op)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        parts = self._xchg("reduce_scatter", inp.detach().clone()) if self.world_size > 1 else [inp]
        n = out.numel()
        acc = torch.zeros_like(out.reshape(-1))
        for p in parts:
            acc.add_(p.reshape(-1)[self.rank * n:(self.rank + 1) * n])
        out.copy_(acc.reshape(out.shape))
        return self._ret(async_op)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        parts = self._xchg("all_gather", inp.detach().clone()) if self.world_size > 1 else [inp]
        out.copy_(torch.cat([p.reshape(-1) for p in parts]).reshape(out.shape))
        return self._ret(async_op)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor):
        parts = self._xchg("all_to_all", inp.detach().clone()) if self.world_size > 1 else [inp]
        outs = list(out.chunk(self.world_size))
        for s, p in enumerate(parts):
            outs[s].copy_(p.chunk(self.world_size)[self.rank])
        return None

    def barrier(self):
        if self.world_size > 1:
            self._xchg("barrier", None)

    def p2p_group(self):
        import contextlib
        return contextlib.nullcontext()  # fake sends are buffered: nothing to pair

    # ------------------------------------------------------ point-to-point
    def send(self, t: torch.Tensor, dst: int):
        if self._enter("send"):
            self.fw.box(self.global_rank, self.ranks[dst]).put(t.detach().clone())
        return None

    def isend(self, t: torch.Tensor, dst: int):
        self.send(t, dst)
        return _Done()

    def recv(self, t: torch.Tensor, src: int):
        self._enter("recv")
        try:
            v = self.fw.box(self.ranks[src], self.global_rank).get(timeout=self.fw.timeout_s)
        except queue.Empty:
            raise CommTimeout(f"recv from rank {src} timed out after {self.fw.timeout_s}s on rank "
                              f"{self.global_rank}") from None
        t.copy_(v.reshape(t.shape))
        return None

    def irecv(self, t: torch.Tensor, src: int):
        self.recv(t, src)
        return _Done()

    # ----------------------------------------------------------- liveness
    def start_heartbeat(self, store=None, period_s: float = 5.0):
        return None

    def stop_heartbeat(self):
        return None

    def dead_ranks(self, timeout_s: float = 30.0, store=None) -> List[int]:
        return sorted({e[1] for e in self.fw.faults.log if e[0] == "kill"})


def run_threads(fn: Callable, world: int, *args, timeout_s: float = 10.0, faults: Optional[FaultPlan] = None,
                return_exceptions: bool = False):
    """Run ``fn(rank, world, comm, *args)`` on ``world`` threads sharing one
    :class:`FakeWorld`.  Returns per-rank results in rank order; with
    ``return_exceptions`` failed ranks yield their exception instead of the
    first one being re-raised."""
    fw = FakeWorld(world, timeout_s, faults)
    res: List[object] = [None] * world
    errs: List[Optional[BaseException]] = [None] * world

    def body(r):
        try:
            res[r] = fn(r, world, fw.communicator(r), *args)
        except BaseException as e:  # noqa: BLE001 - reported to the caller
            errs[r] = e

    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout_s * 20)
    if any(t.is_alive() for t in ts):
        raise CommTimeout("fake ranks did not finish")
    if return_exceptions:
        return [errs[r] if errs[r] is not None else res[r] for r in range(world)]
    for e in errs:
        if e is not None:
            raise e
    return res
