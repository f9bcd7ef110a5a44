"""Native parameter-server mode (reference C25 / C26 / C12 / P7 / P8).

The MI355X training path replaces the reference's ZeroMQ parameter server by
RCCL collectives (:mod:`.distopt`, :mod:`.easgd`).  This module keeps the
reference's *actual* architecture available as well, on the native C++ host
runtime (``_core.PServer`` / ``_core.PSClient``, csrc/runtime/ps.cc):

* :class:`ParamServer` -- one server process role (Server::Run,
  src/server/server.cc:45-214): key-sharded parameters, per-key locks,
  deferred Gets, kStop counting, and the server side of every sync variant:
  EASGD (ElasticParam, src/utils/param.cc:244-258), RandomSync
  (src/utils/param.cc:141-171), the pm prototype's replace-and-return Update
  (src/utils/param.cc:57-61) and a server-side updater (C13 in C++) for
  classic push-gradient / pull-weights training.
* :class:`PSClient` -- the worker side (ParamManager's PS client,
  src/utils/param_manager.cc:103-234, and PMClient Put/Get/Update/Collect,
  src/worker/pm_client.cc:221-287); keys map to servers by ``id % nservers``
  (P7).
* :class:`PSSync` -- drop-in for :class:`.easgd.ElasticSync` /
  :class:`.easgd.RandomSync` that exchanges through the servers: group 0 Puts
  its parameters, the other groups Get them (worker.cc:50-55), then every
  ``sync_frequency`` steps each parameter is sent to its server.

Endpoints: the reference derives them from the hostfile and
``start_port + 1`` (include/utils/cluster.h:80-95); here
:func:`server_endpoints` gives ``host_i:start_port+1+i`` so several servers can
share a host.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch
from ..ops import glue as G


def _core():
    from .. import _core as C  # noqa: N812  (native host runtime)

    return C


def _f32(a: np.ndarray, name: str) -> np.ndarray:
    if not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous):
        raise TypeError(f"{name}: expected a C-contiguous float32 numpy array (written in place)")
    return a


def server_endpoints(nservers: int, start_port: int = 6723, hosts: Optional[Sequence[str]] = None) -> List[str]:
    hosts = list(hosts) if hosts else ["127.0.0.1"]
    return [f"{hosts[i % len(hosts)]}:{start_port + 1 + i}" for i in range(nservers)]


class ParamServer:
    """A parameter-server shard (one process role, or a thread pool inside a
    test).  ``port=0`` binds any free port (see :attr:`port`)."""

    def __init__(self, port: int = 0, nworkers: int = 1):
        self._s = _core().PServer(port, nworkers)

    @property
    def port(self) -> int:
        return self._s.port

    @property
    def messages(self) -> int:
        return self._s.messages

    def set_updater(self, kind: str = "sgd", momentum: float = 0.0, weight_decay: float = 0.0, eps: float = 1e-8,
                    rho: float = 0.9, beta1: float = 0.9, beta2: float = 0.999, method: str = "kFixed",
                    base_lr: float = 0.01, final_lr: float = 0.0, freq: int = 1, gamma: float = 1.0,
                    pow_: float = 0.0) -> None:
        C = _core()
        self._s.set_updater(C.updater_kind(kind), momentum, weight_decay, eps, rho, beta1, beta2, method, base_lr,
                            final_lr, freq, gamma, pow_)

    def set_updater_from_proto(self, up) -> None:
        """UpdaterProto -> server-side updater (param_manager.cc:19-37)."""
        from ..config import schema

        kind = {"kSGD": "sgd_ref", "kNesterov": "nesterov_ref", "kAdaGrad": "adagrad", "kRMSProp": "rmsprop",
                "kAdaDelta": "adadelta"}[schema.enum_name(up, "type")]
        base = up.base_learning_rate if up.HasField("base_learning_rate") else 0.01
        self.set_updater(kind, up.momentum, up.weight_decay, up.delta, up.rho,
                         method=schema.enum_name(up, "learning_rate_change_method"), base_lr=base,
                         final_lr=up.final_learning_rate, freq=up.learning_rate_change_frequency, gamma=up.gamma,
                         pow_=up.pow)

    def wait_stop(self, timeout_s: float = -1.0) -> bool:
        return self._s.wait_stop(timeout_s)

    def value(self, key: int) -> np.ndarray:
        return self._s.value(key)

    def close(self) -> None:
        self._s.close()

    def serve(self, timeout_s: float = -1.0) -> bool:
        """Run until every worker has sent kStop (the server main loop)."""
        ok = self.wait_stop(timeout_s)
        self.close()
        return ok


class PSClient:
    def __init__(self, endpoints: Sequence[str], retries: int = 10, retry_s: float = 0.5):
        self._c = _core().PSClient(list(endpoints), retries, retry_s)

    @property
    def nservers(self) -> int:
        return self._c.nservers

    def put(self, key: int, w: np.ndarray) -> None:
        self._c.put(key, np.ascontiguousarray(w, dtype=np.float32))

    def get(self, key: int, out: np.ndarray) -> int:
        return self._c.get(key, _f32(out, "get"))

    def update(self, key: int, grad: np.ndarray, w_out: np.ndarray, step: int = -1, grad_scale: float = 0.0):
        self._c.update(key, np.ascontiguousarray(grad, dtype=np.float32), _f32(w_out, "update"), step, grad_scale)

    def elastic(self, key: int, w: np.ndarray, alpha: float) -> None:
        """EASGD exchange: server c += alpha (w - c); here w -= alpha (w - c)."""
        self._c.elastic(key, _f32(w, "elastic"), alpha)

    def random_sync(self, key: int, delta: np.ndarray, old_out: np.ndarray, offset: int, stride: int) -> None:
        self._c.random_sync(key, np.ascontiguousarray(delta, dtype=np.float32), _f32(old_out, "random_sync"),
                            int(offset), int(stride))

    def push_replace(self, key: int, w: np.ndarray) -> None:
        self._c.push_replace(key, np.ascontiguousarray(w, dtype=np.float32))

    def push_update(self, key: int, grad: np.ndarray, step: int = -1, grad_scale: float = 0.0) -> None:
        self._c.push_update(key, np.ascontiguousarray(grad, dtype=np.float32), step, grad_scale)

    def collect(self, keys: Sequence[int], outs: Sequence[np.ndarray]) -> int:
        return self._c.collect(list(keys), [_f32(o, "collect") for o in outs])

    def stop(self) -> None:
        self._c.stop()


class PSSync:
    """Worker-side EASGD / RandomSync through native servers (same interface
    as :class:`.easgd.ElasticSync` / :class:`.easgd.RandomSync`).  Parameter
    ``i`` of the flat store is key ``i`` (sharded over servers by
    ``i % nservers``).  Device parameters are mirrored in host memory by a
    native :class:`singa_amd.memory.SyncedBlob` per parameter (the reference
    Param's data blob, src/utils/blob.cc:83-143): a pinned host side synced
    from the store slice before the exchange, written back after it."""

    def __init__(self, store, client: PSClient, group_id: int, ngroups: int, mode: str = "Elastic",
                 moving_rate: float = 0.9, sync_frequency: int = 1, warmup_steps: int = 0, sample_ratio: float = 1.0,
                 seed: int = 1234, key_base: int = 0):
        self.store, self.client = store, client
        self.key_base = int(key_base)  # distinct keys for the partitions of one group
        self.group_id, self.ngroups = group_id, max(1, ngroups)
        self.mode = mode
        self.alpha = moving_rate / self.ngroups  # param_manager.cc:18
        self.sync_frequency = max(1, int(sync_frequency))
        self.warmup_steps = int(warmup_steps)
        self.ratio = float(min(1.0, max(1e-6, sample_ratio)))
        self.seed = seed
        self.nsync = 0
        self._host: List[np.ndarray] = []
        self._snap: List[np.ndarray] = []
        self._blobs = []
        for i, p in enumerate(store.params):
            o, n = store.param_range(i)
            if store.w.is_cuda:
                from ..memory import SyncedBlob
                self._blobs.append(SyncedBlob(None, like=store.w[o:o + n]))
                self._host.append(None)
            else:  # CppCPU: the store slice itself is the host buffer
                self._blobs.append(None)
                self._host.append(store.w[o:o + n].numpy())

    def sync_now(self, step: int) -> bool:
        return step >= self.warmup_steps and (step - self.warmup_steps) % self.sync_frequency == 0

    def _pull_to_host(self, i: int) -> np.ndarray:
        """Host view of parameter i, current with the store (D2H if needed)
        and writable: the exchange updates it in place."""
        b = self._blobs[i]
        if b is None:
            return self._host[i]
        b.cpu_data()  # device -> pinned host when the store holds newer data
        self._host[i] = b.mutable_cpu_data().numpy()
        return self._host[i]

    def _push_from_host(self, i: int) -> None:
        b = self._blobs[i]
        if b is not None:
            b.gpu_data()  # host -> the store slice (stream-ordered)
            b.mutable_gpu_data()  # the device copy is authoritative again (training writes it)

    def _read_host(self, i: int) -> np.ndarray:
        """Read-only host copy of parameter i that leaves the device side
        authoritative: training keeps writing the store slice behind the
        blob's back, so outside an exchange every blob must stay HEAD_AT_GPU
        (else the next sync would read a stale host buffer and push it over
        the trained weights)."""
        b = self._blobs[i]
        if b is None:
            return self._host[i]
        h = b.cpu_data().numpy().copy()  # SYNCED after the D2H copy
        b.mutable_gpu_data()  # SYNCED -> HEAD_AT_GPU (no copy)
        self._host[i] = h
        return h

    def bootstrap(self) -> None:
        """Group 0 Puts every parameter, the other groups Get them (blocking
        until group 0's Put arrived: the server defers the Get)."""
        for i in range(len(self.store.params)):
            if self.group_id == 0:
                self.client.put(self.key_base + i, self._read_host(i))
            else:
                h = self._pull_to_host(i)
                got = self.client.get(self.key_base + i, h)
                if got != h.size:
                    raise RuntimeError(f"PSSync.bootstrap: key {self.key_base + i} holds {got} floats, "
                                       f"parameter {i} has {h.size}")
                self._push_from_host(i)
        self._snap = [h.copy() for h in self._host]
        self.store.sync_low()

    def _progression(self, n: int, step: int):
        m = max(1, int(math.ceil(self.ratio * n)))
        h = (self.seed * 1000003 + step * 7919 + 17) & 0x7FFFFFFF
        offset = h % n
        stride = (h // max(n, 1)) % n or 1
        while math.gcd(stride, n) != 1:
            stride = (stride + 1) % n or 1
        return m, offset, stride

    def sync(self, step: int = 0) -> None:
        if not self._snap:
            self.bootstrap()
        for i in range(len(self.store.params)):
            h = self._pull_to_host(i)
            if self.mode == "RandomSync":
                n = h.size
                m, off, stride = self._progression(n, step)
                idx = (off + np.arange(m, dtype=np.int64) * stride) % n
                delta = h[idx] - self._snap[i][idx]
                old = np.empty(m, dtype=np.float32)
                self.client.random_sync(self.key_base + i, delta, old, off, stride)
                # others' contributions since my last exchange (param.cc:200-229)
                h[idx] += old - self._snap[i][idx]
                self._snap[i][idx] = h[idx]
            else:
                self.client.elastic(self.key_base + i, h, self.alpha)
            self._push_from_host(i)
        self.store.sync_low()
        self.nsync += 1
