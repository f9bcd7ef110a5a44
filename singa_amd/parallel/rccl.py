"""Native RCCL communicator: one process per GPU, collectives over xGMI,
called directly through ``_C.RcclComm`` (csrc/comm/rccl_comm.cpp) -- no
``torch.distributed`` process group in the data path.

Reference mapping: the ZeroMQ Router (C15, src/utils/router.cc:16-123: the
PING/PONG rendezvous, addressed sends) and the ParamManager's Put / Get /
Sync transport (src/utils/param_manager.cc:103-234).  Here:

* rendezvous: rank 0 draws the 128-byte RCCL unique id and publishes it in
  the job's key-value store (the env:// TCP store of torchrun / MASTER_ADDR,
  used only as a KV store); every rank then calls ``ncclCommInitRank``;
* collectives: all_reduce / reduce_scatter / all_gather / broadcast / reduce /
  all_to_all / send / recv.  ``async_op=False`` enqueues on the caller's
  current HIP stream (stream-ordered, HIP-graph capturable); ``async_op=True``
  forks onto the communicator's own high-priority comm stream (fenced by an
  event on the current stream) and returns a handle whose ``wait()`` joins
  the comm stream back into the current stream -- no host blocking, and the
  fork / join is itself capturable, so a training step with bucketed
  all-reduces overlapping the backward can be ONE HIP graph;
* ``split`` = ``ncclCommSplit`` (sub-communicators for layer-partition /
  placement groups);
* ``p2p_group()`` = ``ncclGroupStart/End`` around paired point-to-point calls
  (the pipeline bridges issue a step's sends together with the next receive,
  so crossing 1F1B exchanges cannot deadlock).

``native`` may also be a ``_C.LoopComm`` (csrc/comm/loop_comm.cpp): N ranks as
threads of one process behind the same call surface, on one GPU or on host
memory (:mod:`.loop`), so this wrapper and everything above it run at world
sizes 2..8 before an 8-GPU node is available.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from .. import stream as _stream
from .. import memory as _mem
from ..ops import native as N
from .communicator import Communicator

_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5,
       torch.float64: 6}


class _Done:
    """Completed handle (host-memory loopback ranks finish work eagerly)."""

    def wait(self) -> None:
        return None

    def is_completed(self) -> bool:
        return True

    def synchronize(self) -> None:
        return None


class Work:
    """Handle of an asynchronous collective on the comm stream."""

    __slots__ = ("ev", "keep", "stream")

    def __init__(self, ev, keep, stream: int = 0):
        self.ev = ev
        self.keep = keep  # tensors referenced until the handle is dropped
        self.stream = stream  # the stream the event was recorded on (0: unknown)

    def wait(self) -> None:
        """Stream-ordered: the CURRENT stream waits for the collective (the
        host does not block), like a torch.distributed NCCL work."""
        if not (self.stream and self.stream == _stream.current()):
            self.ev.wait()  # (framework Event: the current stream waits on the device)
        self.keep = None

    def is_completed(self) -> bool:
        return self.ev.query()

    def synchronize(self) -> None:
        self.ev.synchronize()


class RcclCommunicator(Communicator):
    """:class:`Communicator` interface over the native RCCL bindings."""

    capturable = True  # collectives may be captured into a HIP graph

    def __init__(self, world_size: int, rank: int, local_rank: int, store=None, tag: str = "world",
                 native=None, ranks: Optional[List[int]] = None, device: Optional[torch.device] = None):
        super().__init__(world_size, rank, local_rank, "rccl", None, ranks)
        self.loopback = bool(getattr(native, "loopback", False))
        self.host = self.loopback and native.device < 0  # host-memory loopback ranks (CPU CI)
        if self.host:
            self.device = torch.device("cpu")
        else:
            ndev = max(1, torch.cuda.device_count())
            self.device = device or torch.device("cuda", local_rank % ndev)
        self.store = store
        L = N.lib()
        if native is None:
            key = f"singa_amd/rccl_uid/{tag}"
            if rank == 0:
                uid = L.rccl_unique_id()
                if store is not None:
                    store.set(key, uid)
            else:
                if store is None:
                    raise RuntimeError("RcclCommunicator: ranks > 0 need the rendezvous store")
                uid = store.get(key)  # blocks until rank 0 published it
            native = L.RcclComm(bytes(uid), world_size, rank, self.device.index)
        self._c = native
        # high priority: bucket all-reduces issued mid-backward get the CUs
        # they need promptly instead of queueing behind the compute stream
        # (per rank: the loopback world runs several ranks of one process on one GPU)
        self.comm_stream = None if self.host else _stream.pooled(self.device, f"comm-{tag}-r{rank}", priority=-1)
        self.stats = {"calls": 0, "bytes": 0}  # collective calls / payload bytes issued by this rank
        self._group_keep: Optional[list] = None

    @property
    def version(self) -> Optional[int]:
        """librccl version (e.g. 22606 = 2.26.6), the library every rank links."""
        try:
            return int(N.lib().rccl_version())
        except Exception:
            return None

    # ------------------------------------------------------------ plumbing
    def _check(self, *ts):
        for t in ts:
            if t.is_cuda == self.host or not t.is_contiguous():
                raise ValueError("RCCL collectives need dense device tensors" if not self.host else
                                 "host loopback ranks need dense host tensors")
            if t.dtype not in _DT:
                raise TypeError(f"RCCL: unsupported dtype {t.dtype}")
        self.stats["calls"] += 1
        self.stats["bytes"] += sum(t.numel() * t.element_size() for t in ts[:1])

    def _cur(self) -> int:
        return 0 if self.host else N.stream(self.device.index)

    def _run(self, async_op: bool, tensors, fn):
        if not async_op or self.host:
            fn(self._cur())
            return _Done() if async_op else None
        cur = N.stream(self.device.index)
        cs = self.comm_stream
        cs.wait_stream(cur)  # the inputs were produced on the current stream
        fn(cs.cuda_stream)
        if not _stream.is_capturing(cur):
            for t in tensors:  # the caching allocator must not recycle them before the comm stream is done
                _mem.record_stream(t, cs)
        ev = _stream.Event().record(cs)
        return Work(ev, tensors, cs.handle)

    # ---------------------------------------------------------- collectives
    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = False):
        if self.world_size == 1:
            return None
        self._check(t)
        return self._run(async_op, (t,), lambda s: self._c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(),
                                                                      _DT[t.dtype], _OPS[op], s))

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False, op: str = "sum"):
        """inp: flat [world*n] -> out [n] (sum)."""
        if self.world_size == 1:
            if out.data_ptr() != inp.data_ptr():
                from ..ops import glue as G
                G.copy_(out, inp.reshape(out.shape))
            return None
        self._check(out, inp)
        return self._run(async_op, (out, inp), lambda s: self._c.reduce_scatter(
            inp.data_ptr(), out.data_ptr(), out.numel(), _DT[out.dtype], _OPS[op], s))

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """inp [n] -> out flat [world*n]."""
        if self.world_size == 1:
            if out.data_ptr() != inp.data_ptr():
                from ..ops import glue as G
                G.copy_(out, inp.reshape(out.shape))
            return None
        self._check(out, inp)
        return self._run(async_op, (out, inp), lambda s: self._c.all_gather(
            inp.data_ptr(), out.data_ptr(), inp.numel(), _DT[inp.dtype], s))

    def broadcast(self, t: torch.Tensor, src: int = 0, async_op: bool = False):
        if self.world_size == 1:
            return None
        self._check(t)
        return self._run(async_op, (t,), lambda s: self._c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(),
                                                                     _DT[t.dtype], src, s))

    def reduce(self, t: torch.Tensor, dst: int = 0, op: str = "sum", async_op: bool = False):
        if self.world_size == 1:
            return None
        self._check(t)
        return self._run(async_op, (t,), lambda s: self._c.reduce(t.data_ptr(), t.data_ptr(), t.numel(),
                                                                  _DT[t.dtype], _OPS[op], dst, s))

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        if self.world_size == 1:
            if out.data_ptr() != inp.data_ptr():
                from ..ops import glue as G
                G.copy_(out, inp.reshape(out.shape))
            return None
        self._check(out, inp)
        if inp.numel() % self.world_size:
            raise ValueError("all_to_all: numel must divide by the world size")
        return self._run(async_op, (out, inp), lambda s: self._c.all_to_all(
            inp.data_ptr(), out.data_ptr(), inp.numel() // self.world_size, _DT[inp.dtype], s))

    def send(self, t: torch.Tensor, dst: int):
        self._check(t)
        if self._group_keep is not None:
            self._group_keep.append(t)  # grouped calls run at group end: keep the buffer alive until then
        self._c.send(t.data_ptr(), t.numel(), _DT[t.dtype], dst, self._cur())

    def recv(self, t: torch.Tensor, src: int):
        self._check(t)
        if self._group_keep is not None:
            self._group_keep.append(t)
        self._c.recv(t.data_ptr(), t.numel(), _DT[t.dtype], src, self._cur())

    def p2p_group(self):
        """Context manager: the point-to-point calls inside are issued as one
        RCCL group (ncclGroupStart/End) on the current stream."""
        comm = self

        class _G:
            def __enter__(self_):
                comm._group_keep = []
                comm._c.group_start()

            def __exit__(self_, *exc):
                try:
                    comm._c.group_end()
                finally:
                    keep, comm._group_keep = comm._group_keep, None
                    if keep and not comm.host and not _stream.is_capturing():
                        for t in keep:  # the group's kernels run on the current stream
                            _mem.record_stream(t, N.stream(comm.device.index))
                return False
        return _G()

    def isend(self, t: torch.Tensor, dst: int):
        self._check(t)
        return self._run(True, (t,), lambda s: self._c.send(t.data_ptr(), t.numel(), _DT[t.dtype], dst, s))

    def irecv(self, t: torch.Tensor, src: int):
        self._check(t)
        return self._run(True, (t,), lambda s: self._c.recv(t.data_ptr(), t.numel(), _DT[t.dtype], src, s))

    def barrier(self):
        if self.world_size > 1:
            t = torch.zeros(1, dtype=torch.float32, device=self.device)
            self.all_reduce(t)
            if not self.host:
                torch.cuda.current_stream(self.device).synchronize()

    def split(self, ranks: List[int]) -> Optional["RcclCommunicator"]:
        """Collective: every rank of this communicator calls it with the same
        (global-rank) list; members get the sub-communicator (ranks renumbered
        0..len-1 in ascending order), the others None."""
        ranks = sorted(int(r) for r in ranks)
        mine = self.ranks[self.rank] in ranks
        if self.world_size == 1:
            if not mine:
                return None
            c = RcclCommunicator(1, 0, self.local_rank, native=self._c, ranks=ranks, device=self.device)
            c.stats = self.stats
            return c
        sub = self._c.split(0 if mine else -1, ranks.index(self.ranks[self.rank]) if mine else 0)
        if not mine or sub is None:
            return None
        c = RcclCommunicator(sub.nranks, sub.rank, self.local_rank, self.store, native=sub, ranks=ranks,
                             device=self.device)
        c.stats = self.stats  # one traffic account per rank
        return c

    def async_error(self) -> str:
        return self._c.async_error()

    def destroy(self) -> None:
        self.stop_heartbeat()
        self._c.destroy()


def make_store(rank: int, world_size: int, timeout_s: float = 600.0):
    """The job's rendezvous key-value store from the env:// variables
    (MASTER_ADDR / MASTER_PORT; under torchrun the agent's store is reused),
    without creating any torch.distributed process group."""
    import datetime

    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    store, _, _ = next(dist.rendezvous("env://", rank=rank, world_size=world_size,
                                       timeout=datetime.timedelta(seconds=timeout_s)))
    return dist.PrefixStore("singa_amd", store)
