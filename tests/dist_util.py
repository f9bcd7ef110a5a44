"""Multi-process test launcher: spawn ``world`` CPU ranks with the gloo
backend on 127.0.0.1 (the reference tested multi-node over TCP loopback with
real processes; this is the same pattern without ssh)."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, q, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    from singa_amd.parallel import communicator

    communicator.reset()
    try:
        if backend == "rccl":  # the native RCCL communicator (GPU ranks)
            os.environ["SINGA_AMD_COMM"] = "rccl"
            comm = communicator.init_distributed(backend="nccl", timeout_s=120)
        else:
            comm = communicator.init_distributed(backend="gloo", timeout_s=120)
        res = fn(rank, world, comm, *args)
        q.put((rank, "ok", res))
    except Exception:  # report to the parent instead of hanging the others
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
        c = communicator._COMM.get("comm")
        if c is not None and hasattr(c, "destroy"):
            try:
                c.destroy()
            except Exception:
                pass


def run_ranks(fn, world: int = 2, *args, timeout: float = 240.0, backend: str = "gloo"):
    """Run ``fn(rank, world, comm, *args)`` on ``world`` processes; returns
    the per-rank results (must be picklable) in rank order.  backend "rccl":
    GPU ranks over the native RCCL communicator."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q, backend)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    import queue
    import time

    t_end = time.time() + timeout
    try:
        while len(out) < world:
            try:
                rank, status, res = q.get(timeout=1.0)
            except queue.Empty:
                dead = [i for i, p in enumerate(procs) if p.exitcode not in (None, 0) and i not in out]
                if dead:
                    raise RuntimeError(f"ranks {dead} died (exit codes {[procs[i].exitcode for i in dead]})")
                if time.time() > t_end:
                    raise TimeoutError(f"ranks timed out after {timeout}s")
                continue
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{res}")
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [out[r] for r in range(world)]
