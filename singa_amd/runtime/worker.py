"""Worker runtime (reference C24, src/worker/worker.cc): trains a
``ModelProto`` net with the reference cadence semantics.

* nets: train / test / validation built from the same NetProto with phase
  exclusion (worker.cc:69-95); test & validation share the train weights;
* updater from ``UpdaterProto`` (type + the six LR change methods,
  updater.cc:11-182) as a fused flat-buffer optimiser;
* loop: ``warmup_steps`` local steps, bandwidth-model configuration
  (SyncConfig), bootstrap broadcast of group 0's weights, then
  ``train_steps`` with test / validation / display at the configured
  frequencies (include/worker/worker.h:118-158), and EASGD / RandomSync
  exchange every ``sync_frequency`` steps when more than one group runs;
* ``Performance`` accumulates the loss layers' [loss, precision] metric and
  prints averages; ``TimerInfo`` reports ms/step split into forward,
  backward+update and sync (HIP-event timed on a RocmGPU).

One process = one worker group (GPU); ``ClusterProto`` roles map onto
torch.distributed ranks (servers are replaced by collectives).
"""
from __future__ import annotations

import os
import threading
import time
from typing import Callable, Dict, Optional

import numpy as np
import torch

from .. import stream as _stream
from .. import autograd, opt
from ..config import schema
from ..device import Timer, get_default_device
from ..parallel.communicator import Communicator, init_distributed
from ..parallel.easgd import ElasticSync, RandomSync
from ..parallel.ps import PSClient, PSSync, server_endpoints
from ..ops import glue as G
from .neuralnet import NeuralNet


def make_updater(up) -> opt.Optimizer:
    """Updater factory (reference param_manager.cc:19-37)."""
    kind = schema.enum_name(up, "type")
    method = schema.enum_name(up, "learning_rate_change_method")
    base = up.base_learning_rate if up.HasField("base_learning_rate") else 0.01
    sched = opt.RefSchedule(method, base, up.final_learning_rate, up.learning_rate_change_frequency, up.gamma,
                            up.pow)
    if kind == "kSGD":
        return opt.RefSGD(sched, up.momentum, up.weight_decay)
    if kind == "kNesterov":
        return opt.Nesterov(sched, up.momentum, up.weight_decay)
    if kind == "kAdaGrad":
        return opt.AdaGrad(sched, up.delta, up.weight_decay)
    if kind == "kRMSProp":
        return opt.RMSProp(sched, up.rho, up.delta, up.weight_decay)
    if kind == "kAdaDelta":
        return opt.AdaDelta(1.0, up.rho, up.delta, up.weight_decay)
    raise ValueError(kind)


def native_ps_enabled() -> bool:
    """SINGA_AMD_PS=native: exchange through native parameter-server
    processes (``launch --nservers``) instead of RCCL collectives."""
    return os.environ.get("SINGA_AMD_PS", "") == "native"


class Performance:
    def __init__(self, name: str = "train"):
        self.name = name
        self.reset()

    def reset(self):
        self.sum = np.zeros(2)
        self.n = 0

    def update(self, metric: np.ndarray):
        self.sum += metric
        self.n += 1

    def avg(self) -> np.ndarray:
        return self.sum / max(1, self.n)

    def to_string(self) -> str:
        a = self.avg()
        return f"{self.name}: loss : {a[0]:.6f}, precision : {a[1]:.6f}"


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class Worker:
    def __init__(self, model_proto, cluster_proto=None, dev=None, comm: Optional[Communicator] = None,
                 data_override: Optional[dict] = None, log: Callable[[str], None] = print, group_size: int = 1,
                 seed: int = 0, micro_batches: Optional[int] = None, pipeline: Optional[str] = None):
        from .cluster import Cluster

        self.model = model_proto
        self.cluster_proto = cluster_proto
        self.dev = dev or get_default_device()
        self.comm = comm or init_distributed()
        self.cluster = Cluster(cluster_proto, self.comm, make_folders=cluster_proto is not None)
        if self.cluster.nprocs_per_group() > 1:
            group_size = max(group_size, self.cluster.nprocs_per_group())
        self.log = log
        self.group_size = group_size
        self.data_override = data_override or {}
        self.seed = seed
        self.timers = {"forward": 0.0, "backward": 0.0, "sync": 0.0}
        self.history = []
        self.checkpoint_path = ""
        self.checkpoint_every = 0
        # pipelined placed nets (P6): micro-batches per step and the schedule
        self.micro_batches = int(micro_batches or os.environ.get("SINGA_AMD_MICROBATCHES", "1"))
        self.pipeline = pipeline or os.environ.get("SINGA_AMD_PIPELINE", "1f1b")
        if self.comm.world_size > 1:
            # liveness through the rendezvous store (no-op if none is registered)
            self.comm.start_heartbeat()
        self._setup()

    # ------------------------------------------------------------------ setup
    def _phase_has_layers(self, phase: str) -> bool:
        return True

    def _setup(self):
        net = self.model.neuralnet
        cl = self.cluster
        self.group_comm = cl.group_comm if cl.nprocs_per_group() > 1 else None
        self.peer_comm = cl.peer_comm if cl.world > 1 else None
        if self.peer_comm is None and cl.world > 1 and cl.nprocs_per_group() == 1:
            self.peer_comm = self.comm
        # same weights-init seed inside a group (replicas/slices must agree),
        # a different data seed per group
        self.train_net = NeuralNet(net, self.group_size, "kTrain", self.dev, self.data_override,
                                   seed=self.seed + cl.groupid(), comm=self.group_comm)
        self.test_net = None
        self.val_net = None
        eval_group = cl.groupid() == 0  # group 0 tests / validates (worker.h:141-158)
        if self.model.test_steps and self.model.test_frequency and eval_group:
            self.test_net = NeuralNet(net, self.group_size, "kTest", self.dev, self.data_override,
                                      seed=self.seed + 1, comm=self.group_comm)
        if self.model.validation_steps and self.model.validation_frequency and eval_group:
            self.val_net = NeuralNet(net, self.group_size, "kValidation", self.dev, self.data_override,
                                     seed=self.seed + 2, comm=self.group_comm)
        self.updater = make_updater(self.model.updater)
        self.store = self.updater.attach(self.train_net.params())
        for n in (self.test_net, self.val_net):
            if n is not None:
                n.share_weights(self.train_net)
        up = self.model.updater
        self.sync = None
        self.sync_dp = False
        pc = self.peer_comm
        if native_ps_enabled() and cl.nservers() > 0:
            # the reference's own architecture on the native C++ PS (ps.cc):
            # key-sharded servers, Put/Get bootstrap, EASGD / RandomSync
            cp = self.cluster_proto
            port = cp.start_port if cp is not None and cp.HasField("start_port") else 6723
            client = PSClient(server_endpoints(cl.nservers(), port))
            self.sync = PSSync(self.store, client, cl.groupid(), cl.ngroups(), up.param_type or "Elastic",
                               up.moving_rate or 0.9, up.sync_frequency, up.warmup_steps,
                               key_base=65536 * cl.group_procsid())
        elif pc is not None and pc.world_size > 1:
            if cl.synchronous():  # P10: gradient all-reduce across groups every step
                self.sync_dp = True
                pc.broadcast(self.store.w, 0)
                self.store.sync_low()
            elif up.param_type == "RandomSync":
                self.sync = RandomSync(self.store, pc, 1.0, up.sync_frequency, up.warmup_steps)
            else:
                # overlap: on the GPU (native RCCL comm stream) the centre
                # exchange of a sync runs behind the next step's compute
                self.sync = ElasticSync(self.store, pc, up.moving_rate or 0.9, up.sync_frequency,
                                        up.warmup_steps, sharded=cl.sharded_centre(),
                                        overlap=os.environ.get("SINGA_AMD_EASGD_OVERLAP", "1") != "0",
                                        bucket_mb=float(os.environ.get("SINGA_AMD_EASGD_BUCKET_MB", "16")))
        self._setup_executors()
        # per-parameter EASGD schedule (update + exchange per bucket as the
        # backward completes it, joined per layer in the next forward):
        # single-replica, unpartitioned nets with a replicated centre
        self.easgd_pp = (isinstance(self.sync, ElasticSync) and self.sync.per_param_ok()
                         and os.environ.get("SINGA_AMD_EASGD_GRANULARITY", "param") == "param"
                         and len(self.replicas) == 1 and self.micro_batches <= 1 and not self.train_net.dist)
        if self.easgd_pp:
            self.train_net.before_layer = self.sync.wait_params
        self.perf = Performance("train")

    def _setup_executors(self):
        """P3 (reference param_manager.cc:15,163-202, worker.cc:33-39):
        ``nthreads_per_procs`` executor threads, each with its own replica of
        the train net and its own data stream, sharing the weights.  Each
        thread drives its own HIP stream, so small nets overlap on the GPU.
        ``hogwild`` (UpdaterProto, default true): every thread applies its own
        update as soon as its backward is done; otherwise the k gradients are
        summed and ONE update runs with grad_scale = 1/k."""
        k = self.cluster.nthreads_per_procs()
        self.replicas = [self.train_net]
        self.rep_grads = [self.store.g]
        self.hogwild = bool(self.model.updater.hogwild)
        self.streams = None
        if k <= 1:
            return
        if self.train_net.partitioned or self.train_net.placed or self.group_comm is not None:
            raise ValueError("nthreads_per_procs > 1 is supported for unpartitioned nets only")
        for i in range(1, k):
            r = NeuralNet(self.model.neuralnet, 1, "kTrain", self.dev, self.data_override,
                          seed=self.seed + self.cluster.groupid() + 7919 * i)
            g = G.zeros_like(self.store.g)
            r.share_weights_private_grads(self.train_net, self.store, g)
            self.replicas.append(r)
            self.rep_grads.append(g)
        gpu = self.dev.torch_device.type == "cuda"
        self.streams = [_stream.pooled(self.dev.torch_device, f"exec{i}") for i in range(k)] if gpu else None
        # hogwild updates of the SHARED weights/momentum all run on one
        # stream: the lock orders the launches, the single stream serialises
        # the kernels (on per-thread streams they would overlap on the GPU
        # and race their read-modify-write of w and s1)
        self.upd_stream = _stream.pooled(self.dev.torch_device, "update") if gpu else None
        self._upd_lock = threading.Lock()

    # ------------------------------------------------------------- cadence
    @staticmethod
    def _due(step: int, after: int, freq: int) -> bool:
        return freq > 0 and step >= after and (step - after) % freq == 0

    def display_now(self, step):
        return self._due(step, self.model.display_after_steps, self.model.display_frequency)

    def test_now(self, step):
        return self.test_net is not None and step > 0 and self._due(step, self.model.test_after_steps,
                                                                   self.model.test_frequency)

    def validate_now(self, step):
        return self.val_net is not None and step > 0 and self._due(step, self.model.validation_after_steps,
                                                                  self.model.validation_frequency)

    # ---------------------------------------------------------------- steps
    def _thread_step(self, i: int, out: list) -> None:
        net, g = self.replicas[i], self.rep_grads[i]
        ctx = self.streams[i] if self.streams else _Null()
        try:
            with ctx:
                outs = net.forward(training=True)
                roots, seeds = net.backward_roots(outs)
                G.zero_(g)
                if roots:
                    for _ in autograd.backward(roots, seeds):
                        pass
                if self.hogwild:
                    with self._upd_lock:
                        if self.upd_stream is not None:
                            mine = self.streams[i]
                            self.upd_stream.wait_stream(mine)  # this thread's gradient is complete
                            with self.upd_stream:
                                self.updater.update(grad_scale=1.0, g=g)
                            mine.wait_stream(self.upd_stream)  # g is free to be zeroed again
                        else:
                            self.updater.update(grad_scale=1.0, g=g)
                out[i] = net.metrics()
        except BaseException as e:  # surfaced in the caller
            out[i] = e

    def _train_threads(self, step: int) -> np.ndarray:
        k = len(self.replicas)
        if self.streams:
            cur = torch.cuda.current_stream(self.dev.torch_device)
            for s in self.streams:
                s.wait_stream(cur)
        res: list = [None] * k
        with Timer(self.dev) as tb:
            ths = [threading.Thread(target=self._thread_step, args=(i, res)) for i in range(1, k)]
            for t in ths:
                t.start()
            self._thread_step(0, res)
            for t in ths:
                t.join()
            for r in res:
                if isinstance(r, BaseException):
                    raise r
            if self.streams:
                for s in self.streams:
                    _stream.Event().record(s).wait(cur)
            if not self.hogwild:
                for g in self.rep_grads[1:]:
                    G.binary("add", self.store.g, g, out=self.store.g)
                self.updater.update(grad_scale=1.0 / k)
            self.updater.step()
        self.timers["backward"] += tb.ms
        autograd.training = False
        return sum(res) / k

    def train_one_batch(self, step: int) -> np.ndarray:
        if len(self.replicas) > 1:
            m = self._train_threads(step)
            self._maybe_sync(step)
            return m
        net = self.train_net
        if self.micro_batches > 1:
            from ..parallel.pipeline import pipelined_step

            with Timer(self.dev) as tb:
                met = pipelined_step(net, self.store.zero_grad, self.micro_batches, self.pipeline)
                net.sync_replica_grads()
                scale = 1.0
                if self.sync_dp:
                    self.peer_comm.all_reduce(self.store.g)
                    scale = 1.0 / self.peer_comm.world_size
                self.updater.update(grad_scale=scale)
                self.updater.step()
            self.timers["backward"] += tb.ms
            self._maybe_sync(step)
            return met
        with Timer(self.dev) as tf:
            outs = net.forward(training=True)
            roots, seeds = net.backward_roots(outs)
        if self.easgd_pp:
            with Timer(self.dev) as tb:
                self.store.zero_grad()
                es = self.sync
                es.begin_step(self.updater, step)
                if roots:
                    for p, _ in autograd.backward(roots, seeds):
                        es.on_grad(p)  # final: update (and exchange) its bucket now
                net.finish_step()
                es.end_step()
            self.timers["forward"] += tf.ms
            self.timers["backward"] += tb.ms
            autograd.training = False
            return net.metrics()
        with Timer(self.dev) as tb:
            self.store.zero_grad()
            if roots:
                for _ in autograd.backward(roots, seeds):
                    pass
            net.finish_step()
            net.sync_replica_grads()
            scale = 1.0
            if self.sync_dp:
                self.peer_comm.all_reduce(self.store.g)
                scale = 1.0 / self.peer_comm.world_size
            self.updater.update(grad_scale=scale)
            self.updater.step()
        self.timers["forward"] += tf.ms
        self.timers["backward"] += tb.ms
        self._maybe_sync(step)
        autograd.training = False
        return net.metrics()

    def _maybe_sync(self, step: int) -> None:
        if self.sync is not None and self.sync.sync_now(step + 1):
            with Timer(self.dev) as ts:
                if isinstance(self.sync, (RandomSync, PSSync)):
                    self.sync.sync(step)
                else:
                    self.sync.sync()
            self.timers["sync"] += ts.ms

    def test(self, net: NeuralNet, nsteps: int, name: str) -> np.ndarray:
        perf = Performance(name)
        for _ in range(nsteps):
            net.forward(training=False)
            perf.update(net.metrics())
        self.log(f"{perf.to_string()}")
        return perf.avg()

    def timer_info(self, nsteps: int) -> str:
        n = max(1, nsteps)
        return ("time per step: forward {:.2f} ms, backward+update {:.2f} ms, sync {:.2f} ms".format(
            self.timers["forward"] / n, self.timers["backward"] / n, self.timers["sync"] / n))

    def _after_step(self, step: int) -> None:
        """Periodic checkpoint + fault injection (tests of the recovery path:
        SINGA_AMD_FAULT_STEP / SINGA_AMD_FAULT_RANK make that rank die at
        that step unless the run was resumed)."""
        if self.checkpoint_path and self.checkpoint_every and (step + 1) % self.checkpoint_every == 0:
            from .checkpoint import save_worker

            if hasattr(self.sync, "wait"):
                self.sync.wait()  # the centre of an overlapped exchange is part of the checkpoint
            self.step = step + 1
            save_worker(self, self.checkpoint_path.replace("{rank}", str(self.comm.rank)))
        fs = os.environ.get("SINGA_AMD_FAULT_STEP")
        if fs is not None and int(fs) == step and not getattr(self, "start_step", 0):
            if int(os.environ.get("SINGA_AMD_FAULT_RANK", "0")) == self.comm.rank:
                os._exit(17)

    def run(self, train_steps: Optional[int] = None) -> Dict[str, list]:
        steps = train_steps if train_steps is not None else (self.model.train_steps or 0)
        start = int(getattr(self, "start_step", 0))
        warm = min(self.model.updater.warmup_steps if self.sync is not None else 0, steps)
        t0 = time.perf_counter()
        for s in range(start, warm):  # local warm-up (no sync)
            self.step = s
            self.perf.update(self.train_one_batch(s))
        if warm > start and isinstance(self.sync, RandomSync):
            dt = (time.perf_counter() - t0) / (warm - start)
            cp = self.cluster_proto
            bw = cp.bandwidth if cp is not None and cp.HasField("bandwidth") else None
            self.sync.configure_bandwidth(dt, bw)
        if self.sync is not None and not getattr(self.sync, "resumed", False):
            self.sync.bootstrap()
        last = max(warm, start)
        for step in range(max(warm, start), steps):
            self.step = step
            if self.validate_now(step):
                self.history.append(("validation", step, self.test(self.val_net, self.model.validation_steps,
                                                                   "validation")))
            if self.test_now(step):
                self.history.append(("test", step, self.test(self.test_net, self.model.test_steps, "test")))
            self.perf.update(self.train_one_batch(step))
            self._after_step(step)
            if self.display_now(step):
                self.log(f"step-{step} {self.perf.to_string()}")
                self.log(self.timer_info(step - last + 1))
                if self.model.debug:
                    self.log(self.train_net.debug_info())
                self.history.append(("train", step, self.perf.avg()))
                self.perf.reset()
                for k in self.timers:
                    self.timers[k] = 0.0
                last = step + 1
        self.step = steps
        if hasattr(self.sync, "wait"):
            self.sync.wait()
        if isinstance(self.sync, PSSync):
            self.sync.client.stop()  # kStop to every server (param_manager.cc:78-86)
        return {"history": self.history}
