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

from .. import stream as _stream
from .. import memory as _mem
from ..ops import glue as G
from ..ops import native as N
from .communicator import Communicator

XGMI_LINK_GBPS = 153.0  # one MI355X xGMI link, GB/s per direction


def _cpu():
    from ..ops import cpu as CP
    return CP.lib() if CP.enabled() else None


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
    """EASGD over collectives.  Every buffer (the centre or its shard, the
    difference, the gathered centre) is allocated once at bootstrap; the
    worker-side update (w -= d) and the centre update (c += sum d) are native
    kernels on both devices (``easgd_diff`` HIP / CppCPU, native add).

    ``overlap=True`` (GPU, native RCCL communicator): the exchange of step t
    -- reduce-scatter / all-reduce of d, c += sum d, and (sharded) the
    all-gather of the new centre -- is forked onto the communicator's comm
    stream and overlaps step t+1's forward and backward; the next sync joins
    it before reading the centre.  This is the reference's UpdateParam (send
    after the update) / WaitUpdate (receive before the next use) split
    (src/utils/param_manager.cc:163-234) at whole-buffer granularity.  Since
    d_t depends only on w_t and c_t, the overlapped schedule produces the same
    numbers as the synchronous one."""

    def __init__(self, store, comm, moving_rate: float, sync_frequency: int = 1, warmup_steps: int = 0,
                 sharded: bool = False, overlap: bool = False, bucket_mb: float = 16.0):
        super().__init__(store, comm, sync_frequency, warmup_steps)
        self.ngroups = comm.world_size
        self.alpha = moving_rate / max(1, self.ngroups)
        self.sharded = sharded and comm.world_size > 1 and store.numel % comm.world_size == 0
        self.overlap = bool(overlap)
        self.centre: Optional[torch.Tensor] = None
        self._d = self._full = self._shard = None
        self._pending = None  # comm-stream event of the in-flight exchange
        self.bucket_mb = float(bucket_mb)
        self._buckets = None  # per-parameter schedule: [(i0, i1)] store-parameter ranges
        self._bev: list = []  # per bucket: comm-stream event of its in-flight exchange

    def bootstrap(self) -> None:
        super().bootstrap()
        w = self.store.w
        if self.sharded:
            n = self.store.numel // self.comm.world_size
            r = self.comm.rank
            self.centre = _mem.empty(n, dtype=w.dtype, device=w.device)
            G.copy_(self.centre, w[r * n:(r + 1) * n])
            self._shard = _mem.empty_like(self.centre)
            self._full = _mem.empty_like(w)  # the gathered centre the next difference reads
            G.copy_(self._full, w)
        else:
            self.centre = _mem.empty_like(w)
            G.copy_(self.centre, w)
        self._d = _mem.empty_like(w)

    def _can_overlap(self) -> bool:
        return self.overlap and self.store.w.is_cuda and getattr(self.comm, "comm_stream", None) is not None

    def wait(self) -> None:
        """Join every in-flight overlapped exchange into the current stream."""
        if self._pending is not None:
            self._pending.wait()  # the current stream joins the comm stream
            self._pending = None
        for b in range(len(self._bev)):
            self._wait_bucket(b)

    def _ensure_buffers(self) -> None:
        """After a checkpoint restore only the centre is set: rebuild the
        difference buffer and (sharded) the gathered centre -- collectively,
        every rank resumes together."""
        w = self.store.w
        if self._d is None:
            self._d = _mem.empty_like(w)
        if self.sharded and self._full is None:
            self._shard = _mem.empty_like(self.centre)
            self._full = _mem.empty_like(w)
            self.comm.all_gather(self._full, self.centre)

    def sync(self) -> None:
        w = self.store.w
        if self.centre is None:
            self.bootstrap()
        self._ensure_buffers()
        self.wait()  # the previous exchange wrote the centre and read d
        c = self._full if self.sharded else self.centre
        d = self._d
        if w.is_cuda:
            N.lib().easgd_diff(w.data_ptr(), c.data_ptr(), d.data_ptr(), w.numel(), self.alpha, N.stream())
        elif _cpu() is not None and w.dtype == torch.float32 and w.is_contiguous():
            _cpu().easgd_diff(w.data_ptr(), c.data_ptr(), d.data_ptr(), w.numel(), self.alpha)
        else:
            d.copy_(self.alpha * (w - c))
            w.sub_(d)
        self.store.sync_low()  # the worker side is complete: w -= d
        if self._can_overlap():
            cs = self.comm.comm_stream
            cs.wait_stream(torch.cuda.current_stream(w.device))
            with cs:
                self._exchange(d)
            self._pending = _stream.Event().record(cs)
        else:
            self._exchange(d)
        self.nsync += 1

    # -- per-parameter schedule ---------------------------------------------
    # The reference worker updates each parameter as soon as its gradient is
    # final in the backward and sends it to the server right away
    # (Worker::Update -> ParamManager::UpdateParam, src/worker/worker.cc:290-292,
    # src/utils/param_manager.cc:192-201); the parameter's next forward use
    # waits for the reply (WaitUpdate, param_manager.cc:204-234, worker.cc:
    # 249-253).  Here at bucket granularity (contiguous ranges of the flat
    # store, ~bucket_mb each, in backward completion order: the store keeps
    # parameters in reverse creation order): a bucket whose gradients are all
    # final is updated (Optimizer.update_range), its elastic difference taken
    # (w -= d on the range) and its exchange (all-reduce of d, c += sum d)
    # forked onto the comm stream -- overlapping the rest of the backward; the
    # next forward joins each bucket's exchange just before its first layer
    # reads it (NeuralNet.before_layer -> wait_params).  Numerically identical
    # to update + sync() of the whole buffer (every step is elementwise).
    def per_param_ok(self) -> bool:
        return not self.sharded

    def _setup_buckets(self) -> None:
        st = self.store
        lim = max(1, int(self.bucket_mb * (1 << 20) / 4))
        self._buckets, self._pbucket = [], {}
        i0, acc = 0, 0
        for i, p in enumerate(st.params):
            acc += p.data.numel()
            self._pbucket[id(p)] = len(self._buckets)
            if acc >= lim or i == len(st.params) - 1:
                self._buckets.append((i0, i + 1))
                i0, acc = i + 1, 0
        self._bev = [None] * len(self._buckets)

    def _range(self, b: int):
        st = self.store
        i0, i1 = self._buckets[b]
        return st.offsets[i0], (st.offsets[i1] if i1 < len(st.params) else st.numel)

    def begin_step(self, updater, step: int, grad_scale: float = 1.0) -> None:
        """Start a per-parameter step: every bucket is updated (and, when
        this step syncs, exchanged) as its gradients complete (on_grad)."""
        if self._buckets is None:
            self._setup_buckets()
        self._upd, self._gs = updater, grad_scale
        self._syncing = self.sync_now(step + 1)
        # the first sync bootstraps the centre from the UPDATED weights (as
        # sync() after a whole-buffer update does): that step runs whole-buffer
        self._boot = self._syncing and self.centre is None
        if self._boot:
            self._syncing = False
        if self._syncing:
            self._ensure_buffers()
            self.wait()  # (a whole-buffer exchange still in flight)
        self._left = [i1 - i0 for i0, i1 in self._buckets]
        self._done = [False] * len(self._buckets)

    def on_grad(self, p) -> None:
        """The engine yielded p: its gradient is final."""
        b = self._pbucket.get(id(p))
        if b is None or self._done[b]:
            return
        self._left[b] -= 1
        if self._left[b] == 0:
            self._finish(b)

    def _finish(self, b: int) -> None:
        i0, i1 = self._buckets[b]
        self._upd.update_range(i0, i1, self._gs)
        self._done[b] = True
        if not self._syncing:
            return
        o0, o1 = self._range(b)
        self._wait_bucket(b)  # (its previous exchange wrote the centre range read here)
        w, c, d = self.store.w[o0:o1], self.centre[o0:o1], self._d[o0:o1]
        if w.is_cuda:
            N.lib().easgd_diff(w.data_ptr(), c.data_ptr(), d.data_ptr(), w.numel(), self.alpha, N.stream())
        elif _cpu() is not None and w.dtype == torch.float32 and w.is_contiguous():
            _cpu().easgd_diff(w.data_ptr(), c.data_ptr(), d.data_ptr(), w.numel(), self.alpha)
        else:
            d.copy_(self.alpha * (w - c))
            w.sub_(d)
        if self.store.low is not None:
            G.copy_(self.store.low[o0:o1], w)
        if self._can_overlap():
            cs = self.comm.comm_stream
            cs.wait_stream(torch.cuda.current_stream(w.device))
            with cs:
                self.comm.all_reduce(d)
                G.binary("add", c, d, out=c)
            self._bev[b] = _stream.Event().record(cs)
        else:
            self.comm.all_reduce(d)
            G.binary("add", c, d, out=c)

    def end_step(self) -> None:
        """After the backward: buckets whose parameters got no gradient this
        step are updated (and exchanged) now; the optimizer step advances."""
        for b in range(len(self._buckets)):
            if not self._done[b]:
                self._finish(b)
        if self._syncing:
            self.nsync += 1
        self._upd.step()
        if self._boot:
            self.sync()

    def _wait_bucket(self, b: int) -> None:
        ev = self._bev[b]
        if ev is not None:
            ev.wait()
            self._bev[b] = None

    def wait_params(self, params) -> None:
        """A layer is about to read these parameters: join their buckets'
        in-flight exchanges (WaitUpdate)."""
        if not self._bev:
            return
        for p in params:
            b = self._pbucket.get(id(p))
            if b is not None and self._bev[b] is not None:
                self._wait_bucket(b)

    def _exchange(self, d: torch.Tensor) -> None:
        """sum_ranks d -> the centre (and its gathered copy), on the current stream."""
        if self.sharded:
            self.comm.reduce_scatter(self._shard, d)
            G.binary("add", self.centre, self._shard, out=self.centre)
            self.comm.all_gather(self._full, self.centre)
        else:
            self.comm.all_reduce(d)
            G.binary("add", self.centre, d, out=self.centre)


class RandomSync(_SyncBase):
    def __init__(self, store, comm, sample_ratio: float = 1.0, sync_frequency: int = 1, warmup_steps: int = 0,
                 seed: int = 1234):
        super().__init__(store, comm, sync_frequency, warmup_steps)
        self.ratio = float(min(1.0, max(1e-6, sample_ratio)))
        self.seed = seed
        self.snapshot: Optional[torch.Tensor] = None
        self._buf: Optional[torch.Tensor] = None

    def bootstrap(self) -> None:
        super().bootstrap()
        self.snapshot = _mem.empty_like(self.store.w)
        G.copy_(self.snapshot, self.store.w)

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
        if self._buf is None or self._buf.numel() < m:
            self._buf = _mem.empty(m, dtype=torch.float32, device=w.device)
        buf = self._buf[:m]
        if w.is_cuda:
            L = N.lib()
            L.rsync_gather(w.data_ptr(), self.snapshot.data_ptr(), buf.data_ptr(), m, n, a, b, N.stream())
            self.comm.all_reduce(buf)
            L.rsync_scatter(w.data_ptr(), self.snapshot.data_ptr(), buf.data_ptr(), m, n, a, b, N.stream())
        elif _cpu() is not None and w.dtype == torch.float32 and w.is_contiguous():
            C = _cpu()
            C.rsync_gather(w.data_ptr(), self.snapshot.data_ptr(), buf.data_ptr(), m, n, a, b)
            self.comm.all_reduce(buf)
            C.rsync_scatter(w.data_ptr(), self.snapshot.data_ptr(), buf.data_ptr(), m, n, a, b)
        else:
            idx = (b + torch.arange(m, dtype=torch.int64) * a) % n
            buf.copy_(w[idx] - self.snapshot[idx])
            self.comm.all_reduce(buf)
            nv = self.snapshot[idx] + buf
            w[idx] = nv
            self.snapshot[idx] = nv
        self.store.sync_low()
        self.nsync += 1
