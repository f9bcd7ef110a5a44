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
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional

import torch

from .. import stream as _stream
from ..ops import native as N
from .rccl import RcclCommunicator


def run_ranks(fn: Callable, world: int, *args, device: Optional[torch.device] = None, timeout_s: float = 60.0,
              return_exceptions: bool = False) -> List[object]:
    """Run ``fn(rank, world, comm, *args)`` on ``world`` threads sharing one
    loopback world; returns the per-rank results in rank order (re-raising
    the first failure unless ``return_exceptions``).  A failing rank aborts
    the world, so its peers fail fast instead of waiting for the timeout."""
    L = N.lib()
    lw = L.LoopWorld(world, float(timeout_s))
    dev = -1 if device is None or torch.device(device).type == "cpu" else (torch.device(device).index or 0)
    res: List[object] = [None] * world
    errs: List[Optional[BaseException]] = [None] * world

    def body(r: int) -> None:
        native = L.LoopComm(lw, r, dev)
        try:
            if dev >= 0:
                torch.cuda.set_device(dev)
                s = _stream.pooled(torch.device("cuda", dev), f"loop-rank{r}")
                with s:
                    comm = RcclCommunicator(world, r, r, native=native, device=torch.device("cuda", dev))
                    res[r] = fn(r, world, comm, *args)
                s.synchronize()
            else:
                comm = RcclCommunicator(world, r, r, native=native)
                res[r] = fn(r, world, comm, *args)
        except BaseException as e:  # noqa: BLE001 - reported to the caller
            errs[r] = e
            native.abort()

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
