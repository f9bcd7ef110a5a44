"""Benchmarks for the secondary BASELINE.json configs (bench.py covers the
ResNet-50 headline):

* ``mlp_cpu``     -- MLP 784-512-10 on the CppCPU device, SGD, synthetic MNIST (samples/s);
* ``mlp_gpu``     -- the reference's deep-big-simple MLP 784-2500-2000-1500-1000-500-10 on one MI355X;
* ``alexnet``     -- AlexNet (224x224, LRN, dropout) bf16 training, large batch (images/s);
* ``bert``        -- native BERT-base bf16 fine-tuning step, seq 128 (sequences/s);
* ``bert_sonnx``  -- BERT-base exported to ONNX, re-imported with sonnx and
                     fine-tuned through autograd (MatMul/Softmax/LayerNorm) (sequences/s).

Multi-GPU (BASELINE config #4, "AlexNet large-batch on 8x MI355X (bucket
fusion)"): launched under torchrun, ``alexnet`` runs one rank per GPU with
DistOpt over the native RCCL communicator -- per-GPU batch fixed (weak
scaling), ~244 MB of fp32 gradients per step in link-sized buckets overlapped
with the backward -- and rank 0 reports the whole-job images/s (slowest
rank's clock) with the exchange diagnostics:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        tools/bench_suite.py --which alexnet [--grad-dtype bf16] [--bucket-mb 32]

Every step is a full training step (forward, backward, optimizer update);
inputs are synthetic and weights random-init.  One JSON line per benchmark
on stdout (``--out`` appends them to a file too).

    python tools/bench_suite.py --which mlp_cpu,alexnet,bert,bert_sonnx
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


CURVE = []


def _snap(loss):
    """A private fp32 copy of a (graph-static) loss tensor: one native copy
    kernel, no PyTorch kernel in the profiled step."""
    from singa_amd.ops import glue as G
    return G.copy_(torch.empty((), dtype=torch.float32, device=loss.device), G.reshape(loss, ()))


def _time(step, steps, warmup, sync):
    """Times ``steps`` calls after ``warmup``; every step's loss is kept as a
    device tensor (no host sync inside the timed loop) and reported after."""
    CURVE.clear()
    for _ in range(warmup):
        out = step()
        CURVE.append(_snap(out[1].data))
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
        CURVE.append(_snap(out[1].data))
    sync()
    dt = (time.perf_counter() - t0) / steps
    return dt, out


def _rec(name, unit, per_step_items, dt, **cfg):
    curve = [round(float(c), 4) for c in CURVE]
    return {"bench": name, "value": round(per_step_items / dt, 2), "unit": unit, "ms_per_step": round(dt * 1e3, 3),
            "dtype": cfg.pop("dtype", "bf16"), "data": "synthetic, random-init weights", "config": cfg,
            "loss_curve": curve}


def bench_mlp(a, gpu):
    from singa_amd import device, opt, tensor
    from singa_amd.models import mlp

    dev = device.create_rocm_gpu() if gpu else device.get_default_device()
    dev.SetRandSeed(0)
    B = a.batch or (1024 if gpu else 64)
    m = mlp.deep_big_simple() if gpu else mlp.create_model((512,), 10)
    rng = np.random.RandomState(0)
    x = tensor.from_numpy(rng.rand(B, 784).astype(np.float32)).to_device(dev)
    y = tensor.from_numpy(rng.randint(0, 10, B).astype(np.int32)).to_device(dev)
    m.set_optimizer(opt.SGD(0.001, 0.9))  # lr 0.01 diverges for the 6-layer stanh MLP (CPU and GPU alike)
    m.compile([x], is_train=True, use_graph=gpu)
    m.train()
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    dt, (_, loss) = _time(lambda: m(x, y), a.steps, a.warmup, sync)
    name = "mlp_gpu" if gpu else "mlp_cpu"
    host = {"cpus_visible": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
            "omp_threads": os.environ.get("OMP_NUM_THREADS"), "hostname_is_gpu_box": bool(os.environ.get("GRAFT_REPO_ROOT"))}
    model = "MLP 784-2500-2000-1500-1000-500-10 stanh" if gpu else "MLP 784-512-10 relu"
    return _rec(name, "samples/s", B, dt, model=model, batch=B, device="RocmGPU" if gpu else "CppCPU",
                dtype="fp32", optimizer="SGD momentum 0.9", final_loss=round(float(_snap(loss.data)), 4), host=host)


def _world():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def bench_alexnet(a):
    from singa_amd import device, opt, tensor
    from singa_amd.models import alexnet
    from singa_amd.parallel import DistOpt, init_distributed

    world, rank, local = _world()
    if world > 1:
        torch.cuda.set_device(local % torch.cuda.device_count())
        if a.rccl_channels > 0:
            os.environ.setdefault("NCCL_MAX_NCHANNELS", str(a.rccl_channels))
    dev = device.create_rocm_gpu_on(local % max(1, torch.cuda.device_count()), set_default=True)
    dev.SetRandSeed(rank)
    comm = init_distributed(rank=rank, world_size=world, local_rank=local) if world > 1 else None
    B = a.batch or 512
    m = alexnet.create_model(num_classes=1000, compute_dtype=torch.bfloat16)
    rng = np.random.RandomState(rank)
    x = tensor.from_numpy(rng.standard_normal((B, 3, 224, 224)).astype(np.float32)).to_device(dev)
    y = tensor.from_numpy(rng.randint(0, 1000, B).astype(np.int32)).to_device(dev)
    o = opt.SGD(0.01, 0.9, weight_decay=5e-4)
    if comm is not None:
        o = DistOpt(o, comm=comm, bucket_mb=a.bucket_mb, first_bucket_mb=a.first_bucket_mb,
                    grad_dtype=torch.bfloat16 if a.grad_dtype == "bf16" else torch.float32)
        o.time_exposed = a.no_graph  # event timing only in eager mode (not inside a captured graph)
    m.set_optimizer(o)
    m.compile([x], is_train=True, use_graph=not a.no_graph)
    m.train()

    def sync():
        torch.cuda.synchronize()
        if comm is not None:
            comm.barrier()
    dt, (_, loss) = _time(lambda: m(x, y), a.steps, a.warmup, sync)
    extra = {}
    if comm is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev.torch_device)
        comm.all_reduce(t, op="max")
        dt = float(t.item())
        ex = o.exposed_comm_ms()
        extra = {"parallelism": f"dp{world}", "n_gpus": world, "global_batch": world * B,
                 "comm": {"class": type(comm).__name__, "ranks": comm.world_size,
                          "rccl_version": getattr(comm, "version", None), "grad_dtype": a.grad_dtype,
                          "buckets": len(o.buckets), "bucket_mb": a.bucket_mb,
                          "exchange_mb_per_step": round(o.exchange_bytes() / 2**20, 2),
                          "exposed_comm_ms_per_step": None if ex is None else round(ex, 3),
                          "env": {k: os.environ[k] for k in ("NCCL_MAX_NCHANNELS", "NCCL_MIN_NCHANNELS")
                                  if k in os.environ}}}
    rec = _rec("alexnet", "images/s", world * B, dt, model="AlexNet-224 (LRN, dropout 0.5)", batch=B,
               optimizer="SGD momentum 0.9 wd 5e-4", final_loss=round(float(_snap(loss.data)), 4), **extra)
    return rec if rank == 0 else None


def _bert_inputs(dev, B, S, vocab):
    from singa_amd import tensor

    rng = np.random.RandomState(0)
    ids = tensor.from_numpy(rng.randint(0, vocab, (B, S)).astype(np.int64)).to_device(dev)
    y = tensor.from_numpy(rng.randint(0, 2, B).astype(np.int32)).to_device(dev)
    return ids, y


def bench_bert(a):
    from singa_amd import device, opt
    from singa_amd.models import bert

    dev = device.create_rocm_gpu()
    dev.SetRandSeed(0)
    B, S = a.batch or 32, a.seq
    m = bert.bert_base(dropout=0.1, compute_dtype=torch.bfloat16)
    ids, y = _bert_inputs(dev, B, S, 30522)
    m.set_optimizer(opt.Adam(1e-4))
    m.compile([ids], is_train=True, use_graph=not a.no_graph)
    m.train()
    dt, (_, loss) = _time(lambda: m(ids, y), a.steps, a.warmup, torch.cuda.synchronize)
    return _rec("bert", "sequences/s", B, dt, model="BERT-base (native)", batch=B, seq_len=S, optimizer="Adam",
                final_loss=round(float(_snap(loss.data)), 4))


def bench_bert_sonnx(a):
    from singa_amd import device, opt, sonnx
    from singa_amd.models import bert
    from singa_amd.sonnx import onnx_proto as P

    cpu = device.get_default_device()
    cpu.SetRandSeed(0)
    B, S = a.batch or 32, a.seq
    src = bert.bert_base(dropout=0.0, compute_dtype=torch.float32)
    ids_cpu, _ = _bert_inputs(cpu, 2, S, 30522)
    src.compile([ids_cpu], is_train=False)
    blob = sonnx.to_onnx(src, [ids_cpu]).SerializeToString()
    del src
    dev = device.create_rocm_gpu()
    sm = sonnx.SONNXModel(P.load_model(blob), dev, compute_dtype=torch.bfloat16)
    ids, y = _bert_inputs(dev, B, S, 30522)
    sm.set_optimizer(opt.Adam(1e-4))
    sm.compile([ids], is_train=True, use_graph=not a.no_graph)
    sm.train()
    dt, (_, loss) = _time(lambda: sm(ids, y), a.steps, a.warmup, torch.cuda.synchronize)
    return _rec("bert_sonnx", "sequences/s", B, dt, model="BERT-base exported -> ONNX -> sonnx import",
                onnx_bytes=len(blob), batch=B, seq_len=S, optimizer="Adam",
                final_loss=round(float(_snap(loss.data)), 4))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="mlp_cpu,mlp_gpu,alexnet,bert,bert_sonnx")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--out", default="")
    ap.add_argument("--grad-dtype", choices=("fp32", "bf16"), default="fp32")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--first-bucket-mb", type=float, default=4.0)
    ap.add_argument("--rccl-channels", type=int, default=16)
    a = ap.parse_args()
    fns = {"mlp_cpu": lambda: bench_mlp(a, False), "mlp_gpu": lambda: bench_mlp(a, True),
           "alexnet": lambda: bench_alexnet(a), "bert": lambda: bench_bert(a), "bert_sonnx": lambda: bench_bert_sonnx(a)}
    for w in a.which.split(","):
        rec = fns[w]()
        if rec is None:  # non-zero rank of a torchrun job
            continue
        line = json.dumps(rec)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")
        if torch.cuda.is_available():
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
