"""PS-parity microbenchmark.

The reference's only published numbers come from its ``pm`` parameter-server
benchmark (src/test/test_pm.cc, src/worker/pm_client.cc:132-192): each client
thread Puts 12 fp32 tensors shaped like the MNIST MLP 784-2500-2000-1500-1000-
500-10 (47.9 MB), then loops 200 x {Update all 12 -> Collect 12 replies};
published round-trip times are 48.87 ms (1 client thread, 1 server) up to
700.108 ms (16 threads, 1 server), benchmarks/{worker,server}_bottleneck.

On MI355X the same exchange is what a synchronous PS round trip computes:
the 12 gradient tensors live in one flat fp32 buffer, are summed across
ranks with bucketed all-reduce over RCCL/xGMI, and the fused SGD kernel
applies the update to every replica (``mode="allreduce"``); or the elastic
(EASGD, reference ElasticParam) exchange (``mode="easgd"``).

:func:`run` is used by ``tools/ps_bench.py`` and appended (outside the timed
region) to the flagship ``bench.py`` record, so the driver's 1/2/4/8-GPU runs
measure it over real xGMI.
"""
from __future__ import annotations

import time
from typing import Dict

import torch

from ..ops import glue as G

SHAPES = [(784, 2500), (2500,), (2500, 2000), (2000,), (2000, 1500), (1500,), (1500, 1000), (1000,), (1000, 500),
          (500,), (500, 10), (10,)]
# reference ms per update+collect iteration (unspecified CPU cluster, ZeroMQ PS)
BASELINE_MS = {"1 client thread, 1 server": 48.87, "4 clients x 1 thread, 1 server": 172.0,
               "16 threads, 1 server": 700.108, "16 threads, 4 servers": 354.59}


def run(comm, dev, iters: int = 200, warmup: int = 10, mode: str = "allreduce", bucket_mb: float = 32.0) -> Dict:
    from .. import opt
    from ..tensor import Tensor
    from .easgd import ElasticSync

    gpu = dev.torch_device.type == "cuda"
    ps = []
    for s in SHAPES:
        t = Tensor(s, dev, requires_grad=True, stores_grad=True)
        t.gaussian(0.0, 0.01)
        ps.append(t)
    o = opt.SGD(0.01, 0.9)
    st = o.attach(ps)
    nbytes = st.numel * 4
    es = ElasticSync(st, comm, 0.9) if mode == "easgd" else None
    if es is not None:
        es.bootstrap()
    bucket = max(1, int(bucket_mb * (1 << 20) // 4))
    spans = [(s, min(s + bucket, st.numel)) for s in range(0, st.numel, bucket)]

    def one():
        if es is not None:
            es.sync()
            return
        G.random_(st.g, "gaussian", 0.0, 1.0, dev)  # a fresh "gradient" per iteration (the pm client sent random updates)
        hs = [comm.all_reduce(st.g[s:e], async_op=True) for s, e in spans]
        for h in hs:
            if h is not None:
                h.wait()
        o.update(grad_scale=1.0 / comm.world_size)
        o.step()

    def sync():
        if gpu:
            torch.cuda.synchronize()
        comm.barrier()

    for _ in range(warmup):
        one()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        one()
    sync()
    ms = (time.perf_counter() - t0) * 1e3 / iters
    t = torch.tensor([ms], device=dev.torch_device)
    comm.all_reduce(t, op="max")
    ms = float(t.item())
    rec = {"metric": "PS-parity update+collect round trip (12 MLP tensors, 47.9 MB)", "mode": mode,
           "n_ranks": comm.world_size, "device": "gpu" if gpu else "cpu", "iters": iters,
           "ms_per_iter": round(ms, 4), "bytes": nbytes, "algbw_GBps": round(nbytes / (ms * 1e-3) / 1e9, 2)}
    if comm.world_size > 1:
        # a comparison with the reference's networked round trip is only
        # meaningful when the exchange actually crosses ranks
        rec["speedup_vs_reference_1thread_1server"] = round(BASELINE_MS["1 client thread, 1 server"] / ms, 1)
    else:
        rec["note"] = "1 rank: local fused update only, no exchange (not comparable to the reference PS)"
    return rec
