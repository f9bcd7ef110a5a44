"""PS-parity microbenchmark: the reference's ``pm``
benchmark Puts 12 MLP-sized fp32 tensors (47.9 MB, src/worker/pm_client.cc:
132-145) and loops 200 x {Update all 12 -> Collect 12 replies}
(:182-192); published times are 48.87 ms (1 client thread, 1 server) up to
700 ms (16 threads), benchmarks/{worker,server}_bottleneck.

Here an iteration is what replaces that round trip on MI355X:

* ``--mode allreduce`` -- the 12 gradient tensors live in one flat fp32
  buffer; it is summed across ranks with bucketed all-reduce over RCCL/xGMI
  and the fused SGD kernel applies the update (what a synchronous PS round
  trip computes);
* ``--mode easgd`` -- the elastic exchange: fused ``easgd_diff`` kernel,
  all-reduce of the differences, centre update (reference ElasticParam).

Launch with one process per GPU:
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/ps_bench.py
Prints one JSON line (rank 0) with ms/iteration (max over ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = [(784, 2500), (2500,), (2500, 2000), (2000,), (2000, 1500), (1500,), (1500, 1000), (1000,), (1000, 500),
          (500,), (500, 10), (10,)]
BASELINE_MS = {"1 client thread, 1 server": 48.87, "4 clients x 1 thread, 1 server": 172.0,
               "16 threads, 1 server": 700.108, "16 threads, 4 servers": 354.59}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mode", default="allreduce", choices=["allreduce", "easgd"])
    ap.add_argument("--bucket_mb", type=float, default=32.0)
    a = ap.parse_args()
    from singa_amd import device, opt
    from singa_amd.parallel import init_distributed
    from singa_amd.parallel.easgd import ElasticSync
    from singa_amd.tensor import Tensor

    comm = init_distributed()
    gpu = torch.cuda.is_available()
    dev = device.create_rocm_gpu() if gpu else device.get_default_device()
    ps = [Tensor(data=torch.randn(s, device=dev.torch_device) * 0.01, device=dev, requires_grad=True,
                 stores_grad=True) for s in SHAPES]
    o = opt.SGD(0.01, 0.9)
    st = o.attach(ps)
    nbytes = st.numel * 4
    es = ElasticSync(st, comm, 0.9) if a.mode == "easgd" else None
    if es is not None:
        es.bootstrap()
    bucket = max(1, int(a.bucket_mb * (1 << 20) // 4))
    spans = [(s, min(s + bucket, st.numel)) for s in range(0, st.numel, bucket)]

    def one():
        if es is not None:
            es.sync()
            return
        st.g.normal_()  # a fresh "gradient" per iteration (the pm client sent random updates)
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

    for _ in range(a.warmup):
        one()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        one()
    sync()
    ms = (time.perf_counter() - t0) * 1e3 / a.iters
    t = torch.tensor([ms], device=dev.torch_device)
    comm.all_reduce(t, op="max")
    ms = float(t.item())
    if comm.rank == 0:
        print(json.dumps({"metric": "PS-parity update+collect round trip (12 MLP tensors, 47.9 MB)",
                          "mode": a.mode, "n_ranks": comm.world_size, "device": "gpu" if gpu else "cpu",
                          "iters": a.iters, "ms_per_iter": round(ms, 4), "bytes": nbytes,
                          "algbw_GBps": round(nbytes / (ms * 1e-3) / 1e9, 2),
                          "reference_ms (CPU cluster, ZeroMQ PS)": BASELINE_MS}))


if __name__ == "__main__":
    main()
