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

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from singa_amd.parallel import ps_parity  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mode", default="allreduce", choices=["allreduce", "easgd"])
    ap.add_argument("--bucket_mb", type=float, default=32.0)
    a = ap.parse_args()
    from singa_amd import device
    from singa_amd.parallel import init_distributed

    comm = init_distributed()
    dev = device.create_rocm_gpu() if torch.cuda.is_available() else device.get_default_device()
    rec = ps_parity.run(comm, dev, a.iters, a.warmup, a.mode, a.bucket_mb)
    if comm.rank == 0:
        rec["reference_ms (CPU cluster, ZeroMQ PS)"] = ps_parity.BASELINE_MS
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
