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
  placement groups).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from ..ops import native as N
from .communicator import Communicator

_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5,
       torch.float64: 6}


class Work:
    """Handle of an asynchronous collective on the comm stream."""

    __slots__ = ("ev", "keep")

    def __init__(self, ev: torch.cuda.Event, keep):
        self.ev = ev
        self.keep = keep  # tensors referenced until the handle is dropped

    def wait(self) -> None:
        """Stream-ordered: the CURRENT stream waits for the collective (the
        host does not block), like a torch.distributed NCCL work."""
        torch.cuda.current_stream().wait_event(self.ev)
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
        self.comm_stream = torch.cuda.Stream(device=self.device, priority=-1)

    # ------------------------------------------------------------ plumbing
    @staticmethod
    def _check(*ts):
        for t in ts:
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("RCCL collectives need dense device tensors")
            if t.dtype not in _DT:
                raise TypeError(f"RCCL: unsupported dtype {t.dtype}")

    def _run(self, async_op: bool, tensors, fn):
        if not async_op:
            fn(torch.cuda.current_stream(self.device).cuda_stream)
            return None
        cur = torch.cuda.current_stream(self.device)
        cs = self.comm_stream
        cs.wait_stream(cur)  # the inputs were produced on the current stream
        fn(cs.cuda_stream)
        if not torch.cuda.is_current_stream_capturing():
            for t in tensors:  # the caching allocator must not recycle them before the comm stream is done
                t.record_stream(cs)
        ev = torch.cuda.Event()
        ev.record(cs)
        return Work(ev, tensors)

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
        self._c.send(t.data_ptr(), t.numel(), _DT[t.dtype], dst, torch.cuda.current_stream(self.device).cuda_stream)

    def recv(self, t: torch.Tensor, src: int):
        self._check(t)
        self._c.recv(t.data_ptr(), t.numel(), _DT[t.dtype], src, torch.cuda.current_stream(self.device).cuda_stream)

    def isend(self, t: torch.Tensor, dst: int):
        self._check(t)
        return self._run(True, (t,), lambda s: self._c.send(t.data_ptr(), t.numel(), _DT[t.dtype], dst, s))

    def irecv(self, t: torch.Tensor, src: int):
        self._check(t)
        return self._run(True, (t,), lambda s: self._c.recv(t.data_ptr(), t.numel(), _DT[t.dtype], src, s))

    def barrier(self):
        if self.world_size > 1:
            t = torch.empty(1, dtype=torch.float32, device=self.device)
            self.all_reduce(t)
            torch.cuda.current_stream(self.device).synchronize()

    def split(self, ranks: List[int]) -> Optional["RcclCommunicator"]:
        """Collective: every rank of this communicator calls it with the same
        (global-rank) list; members get the sub-communicator (ranks renumbered
        0..len-1 in ascending order), the others None."""
        ranks = sorted(int(r) for r in ranks)
        mine = self.ranks[self.rank] in ranks
        if self.world_size == 1:
            return RcclCommunicator(1, 0, self.local_rank, native=self._c, ranks=ranks,
                                    device=self.device) if mine else None
        sub = self._c.split(0 if mine else -1, ranks.index(self.ranks[self.rank]) if mine else 0)
        if not mine or sub is None:
            return None
        return RcclCommunicator(sub.nranks, sub.rank, self.local_rank, self.store, native=sub, ranks=ranks,
                                device=self.device)

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
