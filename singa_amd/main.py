"""``singa`` entry point (reference C27, src/main.cc:13-62): read the cluster
and model confs, set up the cluster, and run a Worker.  By default servers are
dissolved into collectives, so every process is a worker; with
``launch --nservers N`` (``SINGA_AMD_PS=native``) the extra processes take
the reference's server role (:func:`run_server`: a native C++ parameter
server, csrc/runtime/ps.cc) and the workers exchange through them.

    python -m singa_amd --model_conf examples/mnist/mlp.conf --cluster_conf examples/mnist/cluster.conf

Multi-GPU: one process per GPU, launched by :mod:`singa_amd.launch` (or
``torch.distributed.run``); rank/world come from the environment, and
``--procsID`` is only honoured for single-process runs.  The process picks
GPU ``LOCAL_RANK`` when a GPU is visible, else runs on the CPU.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="singa", description="train a model described by a ModelProto conf")
    ap.add_argument("--procsID", type=int, default=0, help="global process id (single-process runs)")
    ap.add_argument("--hostfile", default="", help="accepted for compatibility; rendezvous is env://")
    ap.add_argument("--cluster_conf", default="", help="ClusterProto text file")
    ap.add_argument("--model_conf", required=True, help="ModelProto text file")
    ap.add_argument("--topology_config", default="", help="Topology text file (pm benchmark)")
    ap.add_argument("--server_threads", type=int, default=1)
    ap.add_argument("--client_threads", type=int, default=1)
    ap.add_argument("--v", type=int, default=0, help="verbosity")
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "gpu"])
    ap.add_argument("--train_steps", type=int, default=None, help="override ModelProto.train_steps")
    ap.add_argument("--synthetic", action="store_true", help="synthetic data for every data layer")
    ap.add_argument("--data_shape", default="28,28", help="synthetic record shape")
    ap.add_argument("--trace", default="", help="write a Chrome trace JSON of per-layer timings here")
    ap.add_argument("--metrics_json", default="", help="append one JSON line per display step here")
    ap.add_argument("--checkpoint", default="", help="save parameters + optimiser state here at the end")
    ap.add_argument("--checkpoint_frequency", type=int, default=0, help="also checkpoint every k steps")
    ap.add_argument("--resume", default="", help="resume from a checkpoint written by --checkpoint")
    ap.add_argument("--micro_batches", type=int, default=None,
                    help="pipelined placed nets: micro-batches per step (singa_amd.parallel.pipeline)")
    ap.add_argument("--pipeline", default=None, choices=["gpipe", "1f1b"], help="pipeline schedule (default 1f1b)")
    return ap


def run_server(model, cluster) -> int:
    """Server role (reference src/main.cc:53-55 -> Server::Run): a native
    parameter-server shard on ``start_port + 1 + server_id`` that serves until
    every worker has sent kStop."""
    from .parallel.ps import ParamServer

    sid = int(os.environ.get("SINGA_AMD_SERVER_ID", "0"))
    nworkers = int(os.environ.get("SINGA_AMD_NWORKERS", "1"))
    start = cluster.start_port if cluster is not None and cluster.HasField("start_port") else 6723
    srv = ParamServer(start + 1 + sid, nworkers)
    srv.set_updater_from_proto(model.updater)
    logging.info("[server %d] listening on port %d for %d workers", sid, srv.port, nworkers)
    srv.serve()
    logging.info("[server %d] has shut down (%d messages)", sid, srv.messages)
    return 0


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    logging.basicConfig(level=logging.DEBUG if a.v >= 3 else logging.INFO, format="%(asctime)s %(message)s")
    from . import device
    from .config import schema
    from .parallel.communicator import init_distributed
    from .runtime import Worker

    model = schema.read_text_file("ModelProto", a.model_conf)
    cluster = schema.read_text_file("ClusterProto", a.cluster_conf) if a.cluster_conf else None
    if a.train_steps is not None:
        model.train_steps = a.train_steps
    if os.environ.get("SINGA_AMD_ROLE") == "server":
        return run_server(model, cluster)
    comm = init_distributed()
    use_gpu = a.device == "gpu" or (a.device == "auto" and device.get_num_gpus() > 0)
    dev = device.create_rocm_gpu() if use_gpu else device.get_default_device()
    rank = comm.rank if comm.world_size > 1 else a.procsID
    log = (lambda s: logging.info("[%d] %s", rank, s))
    if comm.rank == 0:
        log(f"cluster conf:\n{schema.to_text(cluster) if cluster is not None else '(default)'}")
        log(f"model conf:\n{schema.to_text(model)}")
    override = {}
    if a.synthetic:
        shape = tuple(int(x) for x in a.data_shape.split(","))
        override = {"*": {"shape": shape, "nclass": 10}}
        for l in model.neuralnet.layer:
            if l.type in ("kShardData", "kLMDBData"):
                l.type = "kSyntheticData"
    w = Worker(model, cluster, dev=dev, comm=comm, data_override=override, log=log, micro_batches=a.micro_batches,
               pipeline=a.pipeline)
    w.checkpoint_path, w.checkpoint_every = a.checkpoint, a.checkpoint_frequency
    if a.resume:
        from .runtime.checkpoint import load_worker

        load_worker(w, a.resume.replace("{rank}", str(comm.rank)))
        log(f"resumed from {a.resume} at step {w.start_step}")
    tracer = None
    if a.trace:
        from .utils.trace import LayerTracer

        tracer = LayerTracer(w.train_net, dev)
    hist = w.run()
    if tracer is not None:
        tracer.save(a.trace.replace("{rank}", str(comm.rank)))
    if a.metrics_json and comm.rank == 0:
        with open(a.metrics_json, "a") as f:
            for kind, step, m in hist["history"]:
                f.write(json.dumps({"phase": kind, "step": step, "loss": float(m[0]), "precision": float(m[1])})
                        + "\n")
    if a.checkpoint:
        from .runtime.checkpoint import save_worker

        path = a.checkpoint.replace("{rank}", str(comm.rank))
        save_worker(w, path)
        log(f"checkpoint written to {path}")
    log("has shut down")
    return 0


if __name__ == "__main__":
    sys.exit(main())
