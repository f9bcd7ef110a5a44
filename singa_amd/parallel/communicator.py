"""Communicator: one process per GPU, collectives over RCCL/xGMI.

On GPUs :func:`init_distributed` returns the native
:class:`~singa_amd.parallel.rccl.RcclCommunicator` (direct RCCL calls, own
comm stream, HIP-graph capturable).  The ``torch.distributed``-based
:class:`Communicator` below remains for CPU ranks (gloo: the multi-process
tests) and as an explicit fallback (``SINGA_AMD_COMM=torch``).

Replaces the reference's ZeroMQ Router (C15, src/utils/router.cc:16-123:
PING/PONG handshake, addressed sends) and the parameter-server transport
(C25/C26) with ``torch.distributed``:

* rendezvous: the env:// TCP store (MASTER_ADDR/MASTER_PORT, RANK, WORLD_SIZE,
  LOCAL_RANK) replaces the hostfile + procsID roles (X1);
* backend "nccl" (= RCCL on ROCm) for GPU tensors, "gloo" for CPU tests;
* collectives: all_reduce / reduce_scatter / all_gather / broadcast /
  all_to_all / send / recv, with async handles so callers overlap them with
  compute (RCCL runs on its own HIP stream and orders itself against the
  caller's current stream);
* failure detection: a store-based heartbeat and a watchdog timeout on the
  process group (reference had none).

``LocalComm`` is a world-size-1 stand-in used when no process group exists.
"""
from __future__ import annotations

import datetime
import os
import threading
import time
from typing import List, Optional

import torch
import torch.distributed as dist


class Communicator:
    def __init__(self, world_size: int, rank: int, local_rank: int, backend: str, group=None,
                 ranks: Optional[List[int]] = None):
        self.world_size, self.rank, self.local_rank, self.backend = world_size, rank, local_rank, backend
        self.group = group
        self.ranks = list(ranks) if ranks is not None else list(range(world_size))  # local -> global rank
        self._hb_thread = None
        self._hb_stop = threading.Event()

    def split(self, ranks: List[int]) -> Optional["Communicator"]:
        """Sub-communicator over ``ranks`` (global ranks, ascending); every
        rank must call this collectively with the same list.  Returns None
        on non-members.  Ranks inside the sub-communicator are 0..len-1."""
        ranks = sorted(int(r) for r in ranks)
        if self.world_size == 1:
            return Communicator(1, 0, self.local_rank, self.backend) if self.rank in ranks else None
        grp = dist.new_group(ranks=ranks, backend=self.backend) if len(ranks) > 1 else None
        if self.rank not in ranks:
            return None
        if len(ranks) == 1:
            return Communicator(1, 0, self.local_rank, self.backend, None, ranks)
        return Communicator(len(ranks), ranks.index(self.rank), self.local_rank, self.backend, grp, ranks)

    def _g(self, r: int) -> int:
        return self.ranks[r]

    # ---------------------------------------------------------- collectives
    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = False):
        if self.world_size == 1:
            return None
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
               "avg": dist.ReduceOp.SUM}[op]
        if op == "avg" and async_op:
            # the host-side divide cannot follow an async handle: RCCL has a
            # native average; gloo does not, so refuse instead of silently
            # returning the sum
            if self.backend != "nccl":
                raise ValueError("all_reduce(op='avg', async_op=True) needs the nccl (RCCL) backend; "
                                 "use op='sum' and scale, or async_op=False")
            rop = dist.ReduceOp.AVG
        w = dist.all_reduce(t, op=rop, group=self.group, async_op=async_op)
        if op == "avg" and not async_op:
            t.div_(self.world_size)
        return w

    def broadcast(self, t: torch.Tensor, src: int = 0, async_op: bool = False):
        if self.world_size == 1:
            return None
        return dist.broadcast(t, self._g(src), group=self.group, async_op=async_op)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """inp: flat [world*n] -> out [n] (sum)."""
        if self.world_size == 1:
            out.copy_(inp)
            return None
        if self.backend == "gloo":  # gloo has no reduce_scatter_tensor
            tmp = inp.clone()
            dist.all_reduce(tmp, group=self.group)
            n = out.numel()
            out.copy_(tmp[self.rank * n:(self.rank + 1) * n])
            return None
        return dist.reduce_scatter_tensor(out, inp, group=self.group, async_op=async_op)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """inp [n] -> out flat [world*n]."""
        if self.world_size == 1:
            out.copy_(inp)
            return None
        if self.backend == "gloo":
            parts = list(out.chunk(self.world_size))
            dist.all_gather(parts, inp, group=self.group)
            return None
        return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=async_op)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor):
        if self.world_size == 1:
            out.copy_(inp)
            return None
        if self.backend == "gloo":
            ins = list(inp.chunk(self.world_size))
            outs = list(out.chunk(self.world_size))
            outs[self.rank].copy_(ins[self.rank])
            # pairwise exchange through send/recv (gloo lacks all_to_all)
            for k in range(1, self.world_size):
                dst = (self.rank + k) % self.world_size
                src = (self.rank - k) % self.world_size
                s = dist.isend(ins[dst].contiguous(), self._g(dst), group=self.group)
                buf = torch.empty_like(outs[src])
                dist.recv(buf, self._g(src), group=self.group)
                outs[src].copy_(buf)
                s.wait()
            return None
        return dist.all_to_all_single(out, inp, group=self.group)

    def send(self, t: torch.Tensor, dst: int):
        return dist.send(t, self._g(dst), group=self.group)

    def recv(self, t: torch.Tensor, src: int):
        return dist.recv(t, self._g(src), group=self.group)

    def isend(self, t: torch.Tensor, dst: int):
        return dist.isend(t, self._g(dst), group=self.group)

    def irecv(self, t: torch.Tensor, src: int):
        return dist.irecv(t, self._g(src), group=self.group)

    def p2p_group(self):
        """Context manager grouping the point-to-point calls inside (RCCL
        ncclGroupStart/End on the native communicator).  torch.distributed
        sends here are posted as non-blocking isend by the bridges, so no
        grouping is needed: a no-op context."""
        import contextlib
        return contextlib.nullcontext()

    def barrier(self):
        if self.world_size > 1:
            if self.backend == "nccl":
                t = torch.zeros(1, device=torch.device("cuda", torch.cuda.current_device()))
                dist.all_reduce(t, group=self.group)
                torch.cuda.synchronize()
            else:
                dist.barrier(group=self.group)

    # ------------------------------------------------------------ liveness
    def start_heartbeat(self, store=None, period_s: float = 5.0):
        """Every rank bumps ``hb/<rank>`` in the rendezvous store; use
        :meth:`dead_ranks` to find ranks whose heartbeat went stale."""
        store = store or _STORE.get("store")
        if store is None or self._hb_thread is not None:
            return

        def run():
            while not self._hb_stop.wait(period_s):
                try:
                    store.set(f"hb/{self.rank}", str(time.time()))
                except Exception:
                    return
        store.set(f"hb/{self.rank}", str(time.time()))
        self._hb_thread = threading.Thread(target=run, daemon=True)
        self._hb_thread.start()

    def dead_ranks(self, timeout_s: float = 30.0, store=None) -> List[int]:
        store = store or _STORE.get("store")
        if store is None:
            return []
        now, dead = time.time(), []
        for r in range(self.world_size):
            try:
                t = float(store.get(f"hb/{r}").decode())
                if now - t > timeout_s:
                    dead.append(r)
            except Exception:
                dead.append(r)
        return dead

    def stop_heartbeat(self):
        self._hb_stop.set()
        if self._hb_thread is not None:
            self._hb_thread.join(timeout=2.0)
            self._hb_thread = None
        self._hb_stop = threading.Event()


_STORE: dict = {}
_COMM: dict = {}


def init_distributed(rank: Optional[int] = None, world_size: Optional[int] = None,
                     local_rank: Optional[int] = None, backend: Optional[str] = None,
                     timeout_s: float = 600.0) -> Communicator:
    """Initialise (once) the default process group from the environment."""
    if "comm" in _COMM:
        return _COMM["comm"]
    ws = int(world_size if world_size is not None else os.environ.get("WORLD_SIZE", "1"))
    rk = int(rank if rank is not None else os.environ.get("RANK", "0"))
    lr = int(local_rank if local_rank is not None else os.environ.get("LOCAL_RANK", str(rk)))
    if backend is None:
        # SINGA_DIST_BACKEND=gloo rehearses the multi-process GPU path with
        # several ranks sharing one GPU (RCCL refuses two ranks on one device)
        backend = os.environ.get("SINGA_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if (ws > 1 and backend == "nccl" and not dist.is_initialized()
            and os.environ.get("SINGA_AMD_COMM", "rccl") == "rccl"):
        # the native RCCL communicator: the env:// store carries only the
        # unique id and the heartbeats; no torch.distributed process group
        from .rccl import RcclCommunicator, make_store

        torch.cuda.set_device(lr % max(1, torch.cuda.device_count()))
        store = make_store(rk, ws, timeout_s)
        _STORE["store"] = store
        c = RcclCommunicator(ws, rk, lr, store)
        _COMM["comm"] = c
        return c
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend == "nccl":
            torch.cuda.set_device(lr % max(1, torch.cuda.device_count()))
        dist.init_process_group(backend=backend, rank=rk, world_size=ws,
                                timeout=datetime.timedelta(seconds=timeout_s))
    elif dist.is_initialized():
        ws, rk = dist.get_world_size(), dist.get_rank()
        backend = dist.get_backend()
    if ws > 1 and "store" not in _STORE:
        # the rendezvous TCP store of the default group carries the
        # heartbeats (the reference's Router PING/PONG liveness, X1)
        st = default_store()
        if st is not None:
            _STORE["store"] = st
    c = Communicator(ws, rk, lr, backend)
    _COMM["comm"] = c
    return c


def default_store():
    """The default process group's rendezvous store (None if unavailable).
    A PrefixStore keeps heartbeat keys out of the group's own namespace."""
    if not dist.is_initialized():
        return None
    try:
        from torch.distributed import distributed_c10d as c10d

        return dist.PrefixStore("singa_amd", c10d._get_default_store())
    except Exception:
        return None


def register_store(store) -> None:
    """Use ``store`` (any torch.distributed Store) for heartbeats."""
    _STORE["store"] = store


def get_communicator() -> Communicator:
    return _COMM.get("comm") or init_distributed()


def reset():
    c = _COMM.pop("comm", None)
    if c is not None:
        c.stop_heartbeat()
    _STORE.clear()
