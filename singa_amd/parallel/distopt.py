"""Synchronous data parallelism over RCCL with gradient buckets overlapped
with backward.

Reference mapping: the reference ships parameters to a ZeroMQ
parameter server (Put/Get/kSync, src/utils/param_manager.cc:103-234).  On one
MI355X node the PS disappears: every GPU owns a full replica in a flat
:class:`singa_amd.opt.ParamStore`; rank 0's initial weights are broadcast
(X2/X3 -> ncclBroadcast) and gradients are summed with all-reduce (X4).

Buckets are contiguous slices of the flat fp32 gradient buffer.  Because the
store is laid out in reverse creation order, gradients complete front to
back during backward; as soon as every parameter overlapping a bucket is
done, that bucket's all-reduce is forked onto the communicator's comm stream
and overlaps the remaining backward kernels; the fused optimiser update
joins every bucket back in.  Bucket size defaults to 32 MiB: a ring over 8
GPUs moves each bucket in 7 xGMI-link-sized chunks of ~4 MiB, large enough
to run near link bandwidth (§5.8 link-aware sizing), with a smaller first
bucket so communication starts early.

``grad_dtype=torch.bfloat16`` exchanges bf16 buckets (half the xGMI bytes):
each bucket is cast into a bf16 staging buffer, all-reduced, and cast back on
the comm stream.

With the native communicator (:class:`~singa_amd.parallel.rccl.RcclCommunicator`,
the default on GPUs) the fork / join is HIP-graph capturable, so a captured
training step (``Model(use_graph=True)``) contains the overlapped bucket
all-reduces too.  With a communicator that cannot be captured (torch gloo /
NCCL process groups) the collective runs after the replay (:meth:`post_replay`).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from .. import stream as _stream
from .. import memory as _mem
from .. import autograd
from ..ops import functional as F
from ..ops import glue as G
from ..opt import Optimizer, ParamStore
from ..tensor import Tensor
from .communicator import Communicator, init_distributed


class DistOpt:
    def __init__(self, opt: Optimizer, nccl_id=None, local_rank: Optional[int] = None,
                 world_size: Optional[int] = None, rank: Optional[int] = None, bucket_mb: float = 32.0,
                 first_bucket_mb: float = 4.0, overlap: bool = True, comm: Optional[Communicator] = None,
                 grad_dtype: torch.dtype = torch.float32):
        self.opt = opt
        self.comm = comm or init_distributed(rank=rank, world_size=world_size, local_rank=local_rank)
        self.world_size = self.comm.world_size
        self.global_rank = self.rank = self.comm.rank
        self.local_rank = self.comm.local_rank
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.first_bucket_bytes = int(first_bucket_mb * (1 << 20))
        self.overlap = overlap
        self.buckets: List[tuple] = []
        self.graph_mode = False
        self.defer = False
        self.comm_ms = 0.0
        if grad_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("DistOpt: grad_dtype must be float32 or bfloat16")
        self.grad_dtype = grad_dtype
        self._stage = None  # bf16 staging buffer (same layout as the flat gradient)
        # diagnostics: with time_exposed, each step records an event pair
        # around the join of the bucket all-reduces into the compute stream --
        # the GPU time the compute stream waits for communication that the
        # backward did not hide (read with exposed_comm_ms(), after a sync)
        self.time_exposed = False
        self._exposed: List[tuple] = []

    # delegate optimiser attributes (lr, step_counter, store, ...)
    def __getattr__(self, k):
        return getattr(self.__dict__["opt"], k)

    @property
    def store(self) -> Optional[ParamStore]:
        return self.opt.store

    @property
    def step_counter(self):
        return self.opt.step_counter

    @step_counter.setter
    def step_counter(self, v):
        self.opt.step_counter = v

    def attach(self, params: Sequence[Tensor], mixed_bf16: bool = False) -> ParamStore:
        st = self.opt.attach(params, mixed_bf16)
        # rank 0's initial parameters everywhere (reference kPut/kGet bootstrap)
        self.comm.broadcast(st.w, 0)
        st.sync_low()
        self._build_buckets()
        return st

    def _build_buckets(self):
        st = self.store
        self.buckets = []
        start, limit = 0, self.first_bucket_bytes // 4
        cur_params: List[int] = []
        for i, (p, off) in enumerate(zip(st.params, st.offsets)):
            end = off + ((p.data.numel() + 63) // 64 * 64)
            cur_params.append(i)
            if (end - start) >= limit or i == len(st.params) - 1:
                self.buckets.append((start, end, list(cur_params)))
                start, cur_params, limit = end, [], self.bucket_bytes // 4
        self.param_bucket = {}
        for b, (_, _, ps) in enumerate(self.buckets):
            for i in ps:
                self.param_bucket[id(st.params[i])] = b

    def prepare_step(self):
        self.opt.prepare_step()

    def __call__(self, loss: Tensor) -> None:
        self.backward_and_update(loss)

    def backward_and_update(self, loss: Tensor, threshold: int = 0) -> None:
        st = self.store
        if st is None:
            raise RuntimeError("DistOpt: parameters not attached (call model.compile first)")
        st.zero_grad()
        capturing = st.g.is_cuda and _stream.is_capturing()
        capturable = getattr(self.comm, "capturable", False)
        if (capturing and not capturable) or not self.overlap or self.world_size == 1:
            for _ in autograd.backward(loss):
                pass
            if capturing and not capturable:
                self.defer = True  # collective + update happen in post_replay()
                return
            self._allreduce_all()
            self.opt.update(grad_scale=1.0 / self.world_size)
            self.opt.step()
            return
        remaining = [len(ps) for _, _, ps in self.buckets]
        works = []
        for p, _ in autograd.backward(loss):
            b = self.param_bucket.get(id(p))
            if b is None:
                continue
            remaining[b] -= 1
            if remaining[b] == 0:
                works.append(self._reduce_bucket(b))
        for b, r in enumerate(remaining):  # params without gradients this step
            if r > 0:
                works.append(self._reduce_bucket(b))
        ev = None
        if self.time_exposed and torch.cuda.is_available() and self.store.g.is_cuda and not capturing:
            ev = (_stream.Event(timing=True), _stream.Event(timing=True))
            ev[0].record()
        for w in works:
            if w is not None:
                w.wait()
        if ev is not None:
            ev[1].record()
            self._exposed.append(ev)
        self.opt.update(grad_scale=1.0 / self.world_size)
        self.opt.step()

    def exposed_comm_ms(self, reset: bool = True) -> Optional[float]:
        """Mean GPU ms per step the compute stream waited at the bucket joins
        (synchronises on the recorded events)."""
        if not self._exposed:
            return None
        ms = [a.elapsed_time(b) for a, b in self._exposed]
        if reset:
            self._exposed = []
        return sum(ms) / len(ms)

    def exchange_bytes(self) -> int:
        """Bytes one rank contributes to the gradient exchange per step."""
        st = self.store
        return 0 if st is None else st.g.numel() * (2 if self.grad_dtype == torch.bfloat16 else 4)

    def _reduce_bucket(self, b: int):
        """Fork bucket b's all-reduce onto the comm stream (bf16 exchange:
        cast in, all-reduce, cast back -- all on the comm stream)."""
        s, e, _ = self.buckets[b]
        g = self.store.g[s:e]
        if self.grad_dtype == torch.float32 or not g.is_cuda:
            return self.comm.all_reduce(g, async_op=True)
        if self._stage is None or self._stage.numel() != self.store.g.numel():
            self._stage = _mem.empty(self.store.g.numel(), dtype=torch.bfloat16, device=g.device)
        stg = self._stage[s:e]
        cs = getattr(self.comm, "comm_stream", None)
        if cs is None:
            G.copy_(stg, g)
            self.comm.all_reduce(stg)
            G.copy_(g, stg)
            return None
        cs.wait_stream(_stream.current(g.device.index))
        with cs:
            G.copy_(stg, g)  # fp32 -> bf16 (native copy kernel)
            self.comm.all_reduce(stg)  # on the comm stream (its "current" stream here)
            G.copy_(g, stg)
            ev = _stream.Event().record(cs)
        from .rccl import Work
        return Work(ev, (g, stg), cs.handle)

    def _allreduce_all(self):
        if self.world_size == 1:
            return
        works = [self._reduce_bucket(b) for b in range(len(self.buckets))]
        for w in works:
            if w is not None:
                w.wait()

    def post_replay(self) -> None:
        """After a captured forward+backward graph replay: all-reduce + update."""
        if not self.defer:
            return
        self._allreduce_all()
        self.opt.update(grad_scale=1.0 / self.world_size)

    # ------------------------------------------------ SINGA DistOpt extras
    def all_reduce(self, tensor: Tensor) -> None:
        self.comm.all_reduce(tensor.data)

    def fused_all_reduce(self, tensors: Sequence[Tensor], send: bool = True) -> None:
        """One all-reduce over several tensors packed into a flat fp32 buffer
        (native copies in and out)."""
        dev = tensors[0].data.device
        total = sum(t.data.numel() for t in tensors)
        flat = _mem.empty(total, dtype=torch.float32, device=dev)
        o = 0
        for t in tensors:
            n = t.data.numel()
            G.copy_(flat[o:o + n], G.reshape(t.data, (-1,)))
            o += n
        self.comm.all_reduce(flat)
        o = 0
        for t in tensors:
            n = t.data.numel()
            G.copy_(t.data, flat[o:o + n].reshape(t.shape))
            o += n

    def wait(self) -> None:
        if torch.cuda.is_available():
            torch.cuda.current_stream().synchronize()

    def backward_and_partial_update(self, loss: Tensor, threshold: int = 2097152) -> None:
        """SINGA's partial update: all-reduce a rotating window of buckets each
        step (bounded per-step communication), local SGD for the rest."""
        st = self.store
        st.zero_grad()
        for _ in autograd.backward(loss):
            pass
        nb = len(self.buckets)
        k = self.opt.step_counter % max(nb, 1)
        s, e, _ = self.buckets[k]
        self.comm.all_reduce(st.g[s:e])
        G.binary("mul", st.g[s:e], 1.0 / self.world_size, out=st.g[s:e])
        self.opt.update(grad_scale=1.0)
        self.opt.step()

    def backward_and_sparse_update(self, loss: Tensor, threshold: float = 0.01, topK: bool = False,
                                   corr: bool = True) -> None:
        """Sparsified gradient exchange: values with |g| >= threshold (or the
        top threshold-fraction when topK) are summed densely via all-reduce of
        the masked buffer; residuals are kept locally when ``corr``."""
        st = self.store
        st.zero_grad()
        for _ in autograd.backward(loss):
            pass
        g = st.g
        if corr:
            if not hasattr(self, "_resid"):
                self._resid = G.zeros_like(g)
            G.binary("add", g, self._resid, out=g)
        absg = F.unary("abs", g)
        if topK:  # exact k-th largest |g| by on-device radix select (no sort, no host sync)
            thr = G.kth_largest_abs(g, max(1, int(threshold * g.numel())))
        else:
            thr = float(threshold)
        mask = G.binary("ge", absg, thr)
        sparse = G.binary("mul", g, mask)
        if corr:
            G.binary("sub", g, sparse, out=self._resid)
        G.copy_(g, sparse)
        self.comm.all_reduce(g)
        self.opt.update(grad_scale=1.0 / self.world_size)
        self.opt.step()

    def get_states(self):
        return self.opt.get_states()

    def set_states(self, s):
        self.opt.set_states(s)
