#!/usr/bin/env python3
"""Flagship benchmark: ResNet-50 bf16 training throughput (images/s, whole job).

Metric/config from BASELINE.json ("images/sec (whole node) ResNet-50 bf16
training at 1/2/4/8 MI355X"), synthetic ImageNet-shaped data (3x224x224,
1000 classes), random-init weights, full training step timed: forward,
backward, (N>1) bucketed RCCL all-reduce of every gradient, fused SGD-momentum
update of every parameter.

    python bench.py --gpus N --steps K --warmup W     (N > 1: spawns N ranks itself)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Weak scaling: per-GPU batch is fixed (default 1024: sized for the 288 GB of
HBM3E per MI355X -- activations take ~120 GB -- and the larger grids fill the
256 CUs better; see README "Performance" for the measured batch sweep),
global batch = N * 1024.
Rank 0 prints ONE JSON line; value = N * batch * K / max-over-ranks(elapsed).

The other BASELINE.json configs run through the same contract (same JSON
schema, same self-launch, same replica guard):

    --model alexnet   AlexNet-224 (LRN, dropout) bf16, per-GPU batch 512 (config #4 at N = 8)
    --model bert      BERT-base bf16, 32 x 128 tokens per GPU, Adam (config #5, native model)

Replica guard (N > 1): after the timed steps every rank takes per-bucket
float64 checksums (sum |w|, sum w^2) of its fp32 master weights; their max
and min over ranks must agree to 1e-6 relative, else the job exits with code 4
and prints no number (ranks that silently drifted apart would otherwise still
report a throughput).

``--loopback`` runs the N ranks as threads of ONE process on one GPU over the
in-process loopback transport whose all-reduce is captured into the step's
HIP graph (parallel/loop.py WorldGraph): a rehearsal of the N > 1 timed path
(bucket all-reduces forked onto the comm stream inside the captured step) on
a single-GPU box -- its throughput is not a scaling number.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def _load_launcher():
    """singa_amd/launch.py loaded by path: importing the package would load
    the kernel library, and the parent of a self-launched job must stay off
    the GPU (a process that initialised HIP must not fork/exec workers)."""
    import importlib.util

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "singa_amd", "launch.py")
    spec = importlib.util.spec_from_file_location("_singa_amd_launch", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def self_launch(n: int, argv, timeout_s: float = 0.0, script=None) -> int:
    """Run ``script`` (default: this file) as ``n`` ranks with
    RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1/MASTER_PORT set.  The
    children share stdout, so rank 0's JSON line is the job's output; when a
    rank fails the launcher terminates its peers and the failing code is
    returned.  SIGTERM/SIGINT to this parent also stop the children."""
    import signal

    launch = _load_launcher()

    def _stop(signum, frame):
        raise SystemExit(128 + signum)  # unwinds run_job's finally: the children are killed

    signal.signal(signal.SIGTERM, _stop)
    signal.signal(signal.SIGINT, _stop)
    cmd = [sys.executable, "-u", os.path.abspath(script or __file__)]
    rc = launch.run_job(n, list(argv), cmd=cmd, timeout_s=timeout_s)
    if rc < 0:  # a child killed by a signal
        rc = 128 - rc
    if rc != 0:
        print(f"bench.py: self-launched job of {n} ranks failed with exit code {rc}", file=sys.stderr)
    return rc


MODELS = ("resnet50", "resnet18", "resnet101", "resnet152", "alexnet", "bert")


def _build(args, dev, rank: int):
    """(model, inputs, optimizer, record fields) of ``--model``: synthetic
    inputs of the BASELINE config's shape, random-init weights."""
    import torch

    from singa_amd import opt, tensor

    rng = np.random.RandomState(rank)
    name = args.model
    if name.startswith("resnet"):
        from singa_amd.models import resnet

        depth = args.depth or int(name[6:])
        B = args.batch or 1024
        m = resnet.create_model(depth, num_classes=1000, compute_dtype=torch.bfloat16)
        o = opt.SGD(lr=args.lr, momentum=0.9, weight_decay=1e-4)
        x = rng.standard_normal((B, 3, args.image, args.image)).astype(np.float32)
        y = rng.randint(0, 1000, size=(B,)).astype(np.int32)
        inputs = (tensor.from_numpy(x, dev), tensor.from_numpy(y, dev))
        return m, inputs, o, {
            "metric": f"images/sec (whole node) ResNet-{depth} bf16 training", "unit": "images/s", "items": B,
            "batch": B, "model": f"ResNet-{depth}", "seq_len": None, "image": args.image,
            "optimizer": "SGD momentum 0.9 wd 1e-4",
            "data": f"synthetic (random 3x{args.image}x{args.image} images, random labels, random-init weights)"}
    if name == "alexnet":
        from singa_amd.models import alexnet

        B = args.batch or 512
        m = alexnet.create_model(num_classes=1000, compute_dtype=torch.bfloat16)
        o = opt.SGD(lr=args.lr, momentum=0.9, weight_decay=5e-4)
        x = rng.standard_normal((B, 3, 224, 224)).astype(np.float32)
        y = rng.randint(0, 1000, size=(B,)).astype(np.int32)
        inputs = (tensor.from_numpy(x, dev), tensor.from_numpy(y, dev))
        return m, inputs, o, {
            "metric": "images/sec (whole node) AlexNet bf16 training", "unit": "images/s", "items": B, "batch": B,
            "model": "AlexNet-224 (LRN, dropout 0.5)", "seq_len": None, "image": 224,
            "optimizer": "SGD momentum 0.9 wd 5e-4",
            "data": "synthetic (random 3x224x224 images, random labels, random-init weights)"}
    if name == "bert":
        from singa_amd.models import bert

        B, S = args.batch or 32, args.seq
        m = bert.bert_base(dropout=0.1, compute_dtype=torch.bfloat16)
        o = opt.Adam(1e-4)
        ids = rng.randint(0, 30522, (B, S)).astype(np.int64)
        y = rng.randint(0, 2, B).astype(np.int32)
        inputs = (tensor.from_numpy(ids, dev), tensor.from_numpy(y, dev))
        return m, inputs, o, {
            "metric": "sequences/sec (whole node) BERT-base bf16 training", "unit": "sequences/s", "items": B,
            "batch": B, "model": "BERT-base (native, 12 layers, hidden 768)", "seq_len": S, "image": None,
            "optimizer": "Adam",
            "data": f"synthetic (random token ids {B}x{S}, random labels, random-init weights)"}
    raise ValueError(f"unknown --model {name}")


def replica_checksums(optimizer) -> np.ndarray:
    """Per-bucket float64 [sum |w|, sum w^2] of this rank's fp32 master weights
    (one device-to-host copy, outside the timed region)."""
    from singa_amd.ops import glue as G

    w = G.to_numpy(optimizer.store.w).astype(np.float64)
    out = []
    for s, e, _ in (optimizer.buckets or [(0, w.size, None)]):
        seg = w[s:e]
        out += [float(np.abs(seg).sum()), float(np.dot(seg, seg))]
    return np.asarray(out, dtype=np.float64)


def replica_guard(comm, optimizer, dev) -> dict:
    """Max and min over ranks of every checksum; relative spread must be <= 1e-6."""
    from singa_amd.ops import glue as G

    v = replica_checksums(optimizer)
    hi = G.from_numpy(v, dev.torch_device)
    lo = G.from_numpy(v, dev.torch_device)
    comm.all_reduce(hi, op="max")
    comm.all_reduce(lo, op="min")
    hi, lo = G.to_numpy(hi), G.to_numpy(lo)
    rel = np.abs(hi - lo) / np.maximum(np.abs(hi), 1e-30)
    worst = float(rel.max()) if rel.size else 0.0
    return {"checked": True, "buckets": int(v.size // 2), "max_rel_spread": worst, "ok": bool(worst <= 1e-6),
            "bitwise_equal": bool(np.array_equal(hi, lo))}


def run_rank(args, rank: int, world: int, local: int, comm, loopback: bool = False):
    """One rank's benchmark; returns (exit code, JSON record or None)."""
    import torch

    from singa_amd import device
    from singa_amd.ops import glue as G
    from singa_amd.parallel import DistOpt

    # (loopback ranks: every rank thread is on GPU 0)
    dev = device.create_rocm_gpu_on(0 if loopback else local % max(1, torch.cuda.device_count()),
                                    set_default=not loopback)
    if not loopback:
        dev.SetRandSeed(args.seed + rank)
    m, (tx, ty), base_opt, info = _build(args, dev, rank)
    # DistOpt at every N (at N = 1 it is the plain fused update: same path,
    # and the record carries the bucket layout the N > 1 runs exchange)
    optimizer = DistOpt(base_opt, comm=comm, bucket_mb=args.bucket_mb, first_bucket_mb=args.first_bucket_mb,
                        grad_dtype=torch.bfloat16 if args.grad_dtype == "bf16" else torch.float32)
    optimizer.time_exposed = world > 1 and not args.graph
    m.set_optimizer(optimizer)

    # HIP-graph replay of the whole step by default, every N (the round-5
    # ResNet-50 step has ~1 000 launches, many of them few-microsecond BN
    # finalize / tail helpers: replay measured +1.1 % over eager,
    # profiles/r5/ab_graph_vs_eager_r6z.jsonl), so N = 1 and N > 1 time the
    # same path.  With N > 1 each gradient bucket's RCCL all-reduce is forked
    # onto the comm stream inside the captured backward as soon as its
    # gradients are final (the native communicator is capture-safe: RCCL
    # collectives are stream-ordered).  If the capture raises, the model
    # switches to eager execution (Model.graph_fallback) and the record says so.
    m.compile([tx], is_train=True, use_graph=args.graph)
    m.graph_fallback = not loopback  # loopback ranks share one graph: a failure there is a failure
    m.train()

    sync = torch.cuda.synchronize
    for _ in range(args.warmup):
        out, loss = m(tx, ty)
        if args.sync_warmup:
            sync()
    sync()
    if args.warmup > 0:
        # guard against a silently truncated backward (it would inflate the
        # number): after a step every parameter must hold a non-zero gradient
        st = optimizer.store
        norms = G.to_numpy(G.cat([G.reduce(st.g[off:off + p.data.numel()], None, "sumsq").reshape(1)
                                  for p, off in zip(st.params, st.offsets)]))  # native reductions, one copy back
        dead = [i for i in range(len(st.params)) if float(norms[i]) == 0.0]
        if dead:
            names = {id(p): k for k, p in m.get_params().items()}
            print(f"bench.py: {len(dead)} of {len(st.params)} parameters got no gradient: "
                  f"{[names.get(id(st.params[i]), i) for i in dead][:12]}", file=sys.stderr)
            return 3, None
    if world > 1:
        comm.barrier()
    sync()
    t0 = time.perf_counter()
    curve = []
    for _ in range(args.steps):
        out, loss = m(tx, ty)
        if args.loss_curve:
            curve.append(round(float(G.to_numpy(G.to(loss.data, torch.float32))), 4))
    sync()
    if world > 1:
        comm.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    exposed = optimizer.exposed_comm_ms() if world > 1 else None
    replicas = None
    if world > 1:
        t = G.from_numpy(np.array([elapsed, -1.0 if exposed is None else exposed], dtype=np.float64),
                         dev.torch_device)
        comm.all_reduce(t, op="max")
        elapsed, exposed = (float(v) for v in G.to_numpy(t))
        exposed = None if exposed < 0 else exposed  # (only measured eagerly: events inside a graph are not timed)
        replicas = replica_guard(comm, optimizer, dev)
        if not replicas["ok"]:
            if rank == 0:
                print(f"bench.py: replicas diverged across ranks ({replicas}); no number reported", file=sys.stderr)
            return 4, None
    final_loss = float(G.to_numpy(G.to(loss.data, torch.float32)))
    ps = None
    if not args.no_ps_parity and not loopback and info["model"].startswith("ResNet"):
        # the reference's own headline benchmark (PS update+collect of the 12
        # MLP tensors), measured on the same ranks AFTER the
        # timed region: it does not touch the images/s number
        from singa_amd.parallel import ps_parity

        try:
            ps = ps_parity.run(comm, dev, iters=200, warmup=10)
        except Exception as e:  # never lose the timed result to the side benchmark
            ps = {"error": f"{type(e).__name__}: {e}"[:200]}
    ver = getattr(comm, "version", None)
    if ver is None:
        try:
            from singa_amd.ops import native as NN
            ver = int(NN.lib().rccl_version())
        except Exception:
            ver = None
    wg = getattr(comm, "world_graph", None)
    comm_info = {
        "class": type(comm).__name__, "ranks": comm.world_size, "rccl_version": ver,
        "transport": "loopback (in-process ranks on one GPU, captured device all-reduce)" if loopback else
        ("rccl" if world > 1 else None),
        "grad_dtype": args.grad_dtype, "buckets": len(optimizer.buckets), "bucket_mb": args.bucket_mb,
        "first_bucket_mb": args.first_bucket_mb,
        "exchange_mb_per_step": round(optimizer.exchange_bytes() / 2**20, 2),
        "exposed_comm_ms_per_step": None if exposed is None else round(exposed, 3),
        "overlap": "bucket all-reduce forked onto the comm stream during backward",
        "replicas": replicas,
        "env": {k: os.environ[k] for k in ("NCCL_MAX_NCHANNELS", "NCCL_MIN_NCHANNELS", "NCCL_ALGO", "NCCL_PROTO")
                if k in os.environ},
    }
    if wg is not None:
        comm_info["world_graph"] = {"captures": wg.captures, "replays": wg.replays, "nodes": wg.nodes}
    if rank != 0:
        return 0, None
    rate = world * info["items"] * args.steps / elapsed
    base = BASELINE_VALUES.get(info["metric"])
    rec = {
        "metric": info["metric"],
        "value": round(rate, 2),
        "unit": info["unit"],
        "n_gpus": 1 if loopback else world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None if base is None else round(rate / base, 4),
        "dtype": "bf16",
        "data": info["data"],
        "config": {"model": info["model"], "global_batch": world * info["batch"], "seq_len": info["seq_len"],
                   "image": info["image"], "parallelism": f"dp{world}",
                   "exec": "hipgraph" if m.graph_mode else "eager", "optimizer": info["optimizer"],
                   "comm": comm_info, "final_loss": round(final_loss, 4)},
    }
    if loopback:
        rec["loopback_ranks"] = world
        rec["note"] = "rehearsal: N ranks as threads on ONE GPU; not a scaling number"
    if m.graph_error:
        rec["config"]["graph_error"] = m.graph_error
    if curve:
        rec["config"]["loss_curve"] = curve
    if ps is not None:
        rec["ps_parity"] = {k: ps[k] for k in ("ms_per_iter", "algbw_GBps", "n_ranks",
                                               "speedup_vs_reference_1thread_1server", "note", "error")
                            if k in ps}
    return 0, rec


# BASELINE.md publishes no number for these metrics (BASELINE.json "published": {})
BASELINE_VALUES: dict = {}


def _parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", choices=MODELS, default="resnet50",
                    help="resnet50 (the headline), alexnet (config #4), bert (config #5); resnet18/101/152 too")
    ap.add_argument("--batch", type=int, default=0,
                    help="per-GPU batch (default: ResNet 1024 -- fits easily in 288 GB HBM3E and fills the 256 CUs "
                         "better --, AlexNet 512, BERT 32)")
    ap.add_argument("--seq", type=int, default=128, help="BERT sequence length")
    ap.add_argument("--depth", type=int, default=0, help="ResNet depth (overrides --model resnetNN)")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--graph", dest="graph", action="store_true", default=True,
                    help="HIP-graph replay of the whole step (default, every N: +1.1%% over eager launch on the "
                         "round-5 step, profiles/r5/ab_graph_vs_eager_r6z.jsonl; round 3 measured it 0.9%% slower)")
    ap.add_argument("--no-graph", "--eager", dest="graph", action="store_false",
                    help="eager execution (each gradient bucket's all-reduce forked onto the comm stream as soon "
                         "as backward has produced it, as in the captured step)")
    ap.add_argument("--loopback", action="store_true",
                    help="rehearsal: the --gpus N ranks as threads of this process on ONE GPU, all-reduces "
                         "captured into one world graph (parallel/loop.py); not a scaling measurement")
    ap.add_argument("--loss-curve", action="store_true", help="record every step's loss (syncs; diagnostics only)")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--sync-warmup", action="store_true", help="synchronize after every warmup step (diagnostics)")
    ap.add_argument("--no-ps-parity", action="store_true",
                    help="skip the PS-parity microbenchmark appended after the timed region")
    ap.add_argument("--lr", type=float, default=0.01,
                    help="SGD lr (random labels + no warmup: 0.1 occasionally diverges; throughput is lr-independent)")
    ap.add_argument("--grad-dtype", choices=("fp32", "bf16"), default="fp32",
                    help="gradient exchange dtype of the bucketed all-reduce (N > 1)")
    ap.add_argument("--bucket-mb", type=float, default=32.0, help="gradient bucket size (MiB)")
    ap.add_argument("--first-bucket-mb", type=float, default=4.0, help="first (earliest-ready) bucket size (MiB)")
    ap.add_argument("--rccl-channels", type=int, default=16,
                    help="cap on RCCL channels (NCCL_MAX_NCHANNELS) for N > 1; 0 = RCCL's default. The ResNet-50 "
                         "exchange is ~180 MB per GPU per step (~1 ms at 16 channels over the xGMI mesh), so "
                         "fewer channels mainly means fewer CUs taken from the backward it overlaps")
    ap.add_argument("--launch-timeout", type=float, default=0.0,
                    help="self-launch (--gpus N > 1 without WORLD_SIZE): stop the job after this many seconds")
    return ap


def _loopback(args) -> int:
    """--loopback: N rank threads on GPU 0 over the captured loopback world."""
    import torch

    from singa_amd import device
    from singa_amd.parallel.loop import run_ranks

    if not torch.cuda.is_available():
        print("bench.py needs a GPU", file=sys.stderr)
        return 2
    device.create_rocm_gpu_on(0, set_default=True).SetRandSeed(args.seed)
    res = run_ranks(lambda r, w, comm: run_rank(args, r, w, 0, comm, loopback=True), args.gpus,
                    device=torch.device("cuda", 0), timeout_s=600.0, captured=args.graph)
    rc = max(c for c, _ in res)
    if res[0][1] is not None and rc == 0:
        print(json.dumps(res[0][1]), flush=True)
    return rc


def main() -> int:
    args = _parser().parse_args()
    if args.loopback:
        return _loopback(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # self-launch (reference examples/mnist/run.sh:19-30 fans out its own
        # processes): one child rank per GPU; nothing here touches the GPU
        return self_launch(args.gpus, sys.argv[1:], args.launch_timeout)

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"--gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if not torch.cuda.is_available():
        print("bench.py needs a GPU", file=sys.stderr)
        return 2
    torch.cuda.set_device(local % torch.cuda.device_count())
    if world > 1 and args.rccl_channels > 0:
        os.environ.setdefault("NCCL_MAX_NCHANNELS", str(args.rccl_channels))  # before the communicator exists

    from singa_amd.parallel import init_distributed

    comm = init_distributed(rank=rank, world_size=world, local_rank=local)
    rc, rec = run_rank(args, rank, world, local, comm)
    if rec is not None:
        print(json.dumps(rec), flush=True)
    if world > 1:
        if rc == 0:
            comm.barrier()
        if hasattr(comm, "destroy"):
            comm.destroy()
        else:
            import torch.distributed as dist
            dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
