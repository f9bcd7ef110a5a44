"""The reference's ``pm`` parameter-server benchmark on the native PS.

Reference (src/test/test_pm.cc, src/worker/pm_client.cc:132-192): client
threads each Put 12 MLP-shaped fp32 tensors (47.9 MB; one thread Puts, the
others wait), then loop {Update all 12 -> Collect 12 replies}, every request
and reply carrying the full tensor; Update replaces the server's value
(src/utils/param.cc:57-61).  Published per-iteration times:
48.87 ms for 1 client thread / 1 server ... 700.108 ms for 16 threads / 1
server, on an unspecified CPU cluster over ZeroMQ/TCP.

Here: ``nservers`` native servers (csrc/runtime/ps.cc, one handler thread per
connection) and ``clients x threads`` client threads, each with its own
connection to every server, over TCP loopback on this host.  Keys are sharded
by id % nservers (P7).  Prints one JSON line: mean ms per iteration over all
threads, like the reference's tables.

    python tools/pm_bench.py --servers 1 --clients 4 --threads 4 --iters 20
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from singa_amd.parallel.ps import ParamServer, PSClient  # noqa: E402
from singa_amd.parallel.ps_parity import BASELINE_MS, SHAPES  # noqa: E402


def run(nservers: int, nclients: int, nthreads: int, iters: int, warmup: int = 2) -> dict:
    servers = [ParamServer(0, nclients * nthreads) for _ in range(nservers)]
    eps = [f"127.0.0.1:{s.port}" for s in servers]
    nt = nclients * nthreads
    vals = [np.random.RandomState(k).randn(*s).astype(np.float32).ravel() for k, s in enumerate(SHAPES)]
    boot = PSClient(eps)
    for k, v in enumerate(vals):
        boot.put(k, v)
    times = [0.0] * nt
    barrier = threading.Barrier(nt)
    errors = []

    def client(t: int):
        try:
            c = PSClient(eps)
            outs = [np.empty_like(v) for v in vals]
            keys = list(range(len(vals)))
            for it in range(warmup + iters):
                if it == warmup:
                    barrier.wait()
                    t0 = time.perf_counter()
                for k, v in enumerate(vals):
                    c.push_replace(k, v)
                c.collect(keys, outs)
            times[t] = (time.perf_counter() - t0) * 1e3 / iters
            c.stop()
        except Exception as e:  # surfaced below
            errors.append(e)
            barrier.abort()

    ths = [threading.Thread(target=client, args=(t,)) for t in range(nt)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    for s in servers:
        s.close()
    if errors:
        raise errors[0]
    nbytes = sum(v.nbytes for v in vals)
    return {"metric": "pm update+collect per iteration (12 MLP tensors, 47.9 MB, native PS over TCP loopback)",
            "servers": nservers, "clients": nclients, "threads_per_client": nthreads, "iters": iters,
            "ms_per_iter": round(float(np.mean(times)), 2), "ms_max": round(float(np.max(times)), 2),
            "bytes_each_way": nbytes}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--servers", type=int, default=1)
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sweep", action="store_true", help="the reference's table: servers 1/2/4 x 1/4/16 threads")
    a = ap.parse_args()
    if not a.sweep:
        rec = run(a.servers, a.clients, a.threads, a.iters)
        rec["reference_ms"] = BASELINE_MS
        print(json.dumps(rec), flush=True)
        return
    for nserv in (1, 2, 4):
        for (nc, nth) in ((1, 1), (4, 1), (4, 4)):
            print(json.dumps(run(nserv, nc, nth, a.iters)), flush=True)


if __name__ == "__main__":
    main()
