"""Inter-group parameter synchronisation without a parameter server.

* :class:`ElasticSync` -- Elastic Averaging SGD (reference P1, ElasticParam,
  src/utils/param.cc:244-284).  The reference server computed
  d = alpha*(w_worker - c), c += d, and the worker applied w -= d, with
  alpha = moving_rate / ngroups (src/utils/param_manager.cc:18).  Here every
  rank holds the centre c (replicated, or sharded with reduce-scatter /
  all-gather for large models): each rank computes its elastic difference
  d_i with one fused HIP kernel (``easgd_diff``: w -= d), the d_i are summed
  by an all-reduce over RCCL/xGMI, and c += sum_i d_i -- exactly the state a
  PS would reach after receiving every group's message.
* :class:`RandomSync` -- bandwidth-adaptive random-sample exchange (P2,
  src/utils/param.cc:130-241).  All ranks derive the SAME index sample from a
  shared (step-derived) seed -- an arithmetic progression with a stride
  coprime to n, so no duplicates and no index traffic -- gather
  w - snapshot on those indices (``rsync_gather`` kernel), all-reduce the
  compact buffer, and scatter snapshot + sum back (``rsync_scatter``).
  ``sample_ratio`` comes from the reference's bandwidth model
  (param_manager.cc:88-96) with the xGMI bandwidth instead of 100 MB/s.

Both run on flat :class:`singa_amd.opt.ParamStore` buffers, every
``sync_frequency`` steps after ``warmup_steps``.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..ops import native as N
from .communicator import Communicator

XGMI_LINK_GBPS = 153.0  # one MI355X xGMI link, GB/s per direction


class _SyncBase:
    def __init__(self, store, comm: Communicator, sync_frequency: int = 1, warmup_steps: int = 0):
        self.store, self.comm = store, comm
        self.sync_frequency = max(1, int(sync_frequency))
        self.warmup_steps = int(warmup_steps)
        self.nsync = 0

    def sync_now(self, step: int) -> bool:
        """Reference SyncNow (param_manager.cc:158-162)."""
        return step >= self.warmup_steps and (step - self.warmup_steps) % self.sync_frequency == 0

    def bootstrap(self) -> None:
        """Group 0's parameters everywhere (kPut by group 0, kGet by the rest)."""
        self.comm.broadcast(self.store.w, 0)
        self.store.sync_low()


class ElasticSync(_SyncBase):
    def __init__(self, store, comm, moving_rate: float, sync_frequency: int = 1, warmup_steps: int = 0,
                 sharded: bool = False):
        super().__init__(store, comm, sync_frequency, warmup_steps)
        self.ngroups = comm.world_size
        self.alpha = moving_rate / max(1, self.ngroups)
        self.sharded = sharded and comm.world_size > 1 and store.numel % comm.world_size == 0
        self.centre: Optional[torch.Tensor] = None

    def bootstrap(self) -> None:
        super().bootstrap()
        if self.sharded:
            n = self.store.numel // self.comm.world_size
            r = self.comm.rank
            self.centre = self.store.w[r * n:(r + 1) * n].clone()
        else:
            self.centre = self.store.w.clone()

    def sync(self) -> None:
        w = self.store.w
        if self.centre is None:
            self.bootstrap()
        if self.sharded:
            full_c = torch.empty_like(w)
            self.comm.all_gather(full_c, self.centre)
            c = full_c
        else:
            c = self.centre
        d = torch.empty_like(w)
        if w.is_cuda:
            N.lib().easgd_diff(w.data_ptr(), c.data_ptr(), d.data_ptr(), w.numel(), self.alpha, N.stream())
        else:
            d.copy_(self.alpha * (w - c))
            w.sub_(d)
        if self.sharded:
            shard = torch.empty_like(self.centre)
            self.comm.reduce_scatter(shard, d)
            self.centre.add_(shard)
        else:
            self.comm.all_reduce(d)
            self.centre.add_(d)
        self.store.sync_low()
        self.nsync += 1


class RandomSync(_SyncBase):
    def __init__(self, store, comm, sample_ratio: float = 1.0, sync_frequency: int = 1, warmup_steps: int = 0,
                 seed: int = 1234):
        super().__init__(store, comm, sync_frequency, warmup_steps)
        self.ratio = float(min(1.0, max(1e-6, sample_ratio)))
        self.seed = seed
        self.snapshot: Optional[torch.Tensor] = None

    def bootstrap(self) -> None:
        super().bootstrap()
        self.snapshot = self.store.w.clone()

    def configure_bandwidth(self, step_seconds: float, bandwidth_mbps: Optional[float] = None,
                            nservers: int = 1) -> float:
        """sample_ratio = bandwidth*nservers / (modelMB*nworkers/t), capped at 1."""
        bw = bandwidth_mbps if bandwidth_mbps is not None else XGMI_LINK_GBPS * 1e3
        model_mb = self.store.numel * 4 / 1e6
        need = model_mb * self.comm.world_size / max(step_seconds, 1e-9)
        self.ratio = float(min(1.0, bw * max(1, nservers) / max(need, 1e-9)))
        return self.ratio

    def _progression(self, n: int, step: int):
        m = max(1, int(math.ceil(self.ratio * n)))
        h = (self.seed * 1000003 + step * 7919 + 17) & 0x7FFFFFFF
        b = h % n
        a = (h // max(n, 1)) % n or 1
        while math.gcd(a, n) != 1:
            a = (a + 1) % n or 1
        return m, a, b

    def sync(self, step: int = 0) -> None:
        w = self.store.w
        if self.snapshot is None:
            self.bootstrap()
        n = w.numel()
        m, a, b = self._progression(n, step)
        buf = torch.empty(m, dtype=torch.float32, device=w.device)
        if w.is_cuda:
            L = N.lib()
            L.rsync_gather(w.data_ptr(), self.snapshot.data_ptr(), buf.data_ptr(), m, n, a, b, N.stream())
            self.comm.all_reduce(buf)
            L.rsync_scatter(w.data_ptr(), self.snapshot.data_ptr(), buf.data_ptr(), m, n, a, b, N.stream())
        else:
            idx = (b + torch.arange(m, dtype=torch.int64) * a) % n
            buf.copy_(w[idx] - self.snapshot[idx])
            self.comm.all_reduce(buf)
            nv = self.snapshot[idx] + buf
            w[idx] = nv
            self.snapshot[idx] = nv
        self.store.sync_low()
        self.nsync += 1
