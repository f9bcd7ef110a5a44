"""``singa_amd.opt`` -- optimisers, LR schedules and the flat ParamStore.

:class:`ParamStore` is the MI355X form of the reference's ParamManager
(C14, src/utils/param_manager.cc:40-69), which carved every local parameter
out of ONE contiguous float buffer.  Here the store owns

* ``w``   fp32 master weights (flat), every param's ``.data`` is a view;
* ``g``   fp32 gradients (flat), every param's ``.grad_view``;
* ``low`` optional bf16 compute copy (flat), every param's ``.low``;
* ``s1``/``s2`` optimiser state,

laid out in *reverse* creation order, so gradients -- produced last-layer
first during backward -- fill the buffer front to back and contiguous
all-reduce buckets complete in order (see :mod:`singa_amd.parallel.distopt`).
4-D conv weights use channels_last views on the GPU, i.e. the flat memory is
[K][R][S][C], exactly what the implicit-GEMM kernels read and the weight-
gradient kernel writes.

One fused HIP launch (``csrc/kernels/optim.hip``) updates every parameter;
lr and the step counter live in a device tensor so the update can sit inside a
captured HIP graph while the host changes the schedule.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

from . import autograd, memory
from .ops import glue as G
from .ops import native as N
from .tensor import Tensor

ALIGN = 64  # elements; keeps every param view 256-B aligned
# skip zeroing gradient slices whose producer overwrites them (ParamStore.zero_grad)
LAZY_ZERO = True


# ---------------------------------------------------------------------------
# learning-rate schedules (reference UpdaterProto change methods,
# src/utils/updater.cc:11-51, plus SINGA's DecayScheduler API)
# ---------------------------------------------------------------------------
class DecayScheduler:
    def __init__(self, init_value: float):
        self.init_value = float(init_value)

    def __call__(self, step: int) -> float:
        raise NotImplementedError


class Constant(DecayScheduler):
    def __call__(self, step):
        return self.init_value


class ExponentialDecay(DecayScheduler):
    def __init__(self, init_value, decay_steps, decay_rate, staircase=False):
        super().__init__(init_value)
        self.decay_steps, self.decay_rate, self.staircase = decay_steps, decay_rate, staircase

    def __call__(self, step):
        e = step / self.decay_steps
        if self.staircase:
            e = math.floor(e)
        return self.init_value * self.decay_rate ** e


class RefSchedule(DecayScheduler):
    """The reference's six ChangeProto methods (kFixed, kInverse_t, kInverse,
    kExponential, kLinear, kStep)."""

    def __init__(self, method: str, base: float, final: float = 0.0, freq: int = 1, gamma: float = 1.0,
                 pow_: float = 0.0):
        super().__init__(base)
        self.method, self.final, self.freq, self.gamma, self.pow = method, final, max(1, freq), gamma, pow_

    def __call__(self, step):
        b, m = self.init_value, self.method
        if m == "kFixed":
            return b
        if m == "kLinear":
            r = step / self.freq
            return (1 - r) * b + r * self.final if r < 1 else self.final
        if m == "kExponential":
            return b / (2.0 ** (step / self.freq))
        if m == "kInverse_t":
            return b / (1.0 + step / self.final)
        if m == "kInverse":
            return b * (1.0 + self.gamma * step) ** (-self.pow)
        if m == "kStep":
            return b * self.gamma ** (step // self.freq)
        raise ValueError(m)


def _sched(lr) -> DecayScheduler:
    return lr if isinstance(lr, DecayScheduler) else Constant(lr)


# ---------------------------------------------------------------------------
def _native_cpu():
    """The host runtime module (_core) if built: its C++ updaters run the
    CppCPU optimiser step (the torch expression in Optimizer._cpu_update is
    the reference oracle of the tests)."""
    global _CORE
    if _CORE is None:
        try:
            from . import _core as C  # noqa: N812

            _CORE = C if hasattr(C, "opt_update") else False
        except Exception:
            _CORE = False
    return _CORE or None


_CORE = None


class ParamStore:
    def __init__(self, params: Sequence[Tensor], mixed_bf16: bool = False, reverse: bool = True,
                 state_slots: int = 2, channels_last: Optional[bool] = None):
        seen, ps = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                ps.append(p)
        self.params: List[Tensor] = list(reversed(ps)) if reverse else ps
        assert self.params, "ParamStore needs at least one parameter"
        dev = self.params[0].data.device
        self.device = dev
        self.gpu = dev.type == "cuda"
        # flat memory of 4-D weights: [K][R][S][C] for the GPU kernels, [K][C][R][S] on the CPU
        self.channels_last = self.gpu if channels_last is None else bool(channels_last)
        self.offsets, off = [], 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.data.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        # the flat buffers live in the framework's own memory pools (HBM caching
        # pool / aligned host pool, singa_amd/memory.py), not PyTorch's allocator
        self.w = memory.zeros((off,), torch.float32, dev)
        self.g = memory.zeros((off,), torch.float32, dev)
        self.low = memory.zeros((off,), torch.bfloat16, dev) if mixed_bf16 else None
        self.s1 = memory.zeros((off,), torch.float32, dev) if state_slots >= 1 else None
        self.s2 = memory.zeros((off,), torch.float32, dev) if state_slots >= 2 else None
        self.mixed = mixed_bf16
        for p, o in zip(self.params, self.offsets):
            n = p.data.numel()
            src = p.data.detach()
            wv = self._view(self.w, o, p.data.shape)
            G.copy_(wv, src)
            p.data = wv
            p.grad_view = self._view(self.g, o, p.data.shape)
            if self.low is not None:
                p.low = self._view(self.low, o, p.data.shape)
                G.copy_(p.low, wv)
        self._build_chunks()

    def _view(self, flat: torch.Tensor, off: int, shape) -> torch.Tensor:
        n = int(np.prod(shape)) if len(shape) else 1
        v = flat[off:off + n]
        if len(shape) == 4 and self.channels_last:
            K, C, R, S = shape
            return v.view(K, R, S, C).permute(0, 3, 1, 2)  # logical KCRS, memory KRSC
        return v.view(*shape) if len(shape) else v.view(())

    def _build_chunks(self, chunk: int = 16384):
        starts, lens, segs = [], [], []
        lrm, wdm = [], []
        self.chunk_lo = []  # first chunk of each parameter (update_range)
        for i, (p, o) in enumerate(zip(self.params, self.offsets)):
            self.chunk_lo.append(len(starts))
            meta = p.param_meta or {}
            lrm.append(float(meta.get("lr_mult", 1.0)))
            wdm.append(float(meta.get("wd_mult", 1.0)))
            n = p.data.numel()
            for s in range(0, n, chunk):
                starts.append(o + s)
                lens.append(min(chunk, n - s))
                segs.append(i)
        dev = self.device
        self.nchunks = len(starts)
        self.cstart = torch.tensor(starts, dtype=torch.int64, device=dev)
        self.clen = torch.tensor(lens, dtype=torch.int32, device=dev)
        self.cseg = torch.tensor(segs, dtype=torch.int32, device=dev)
        self.seg_lr = torch.tensor(lrm, dtype=torch.float32, device=dev)
        self.seg_wd = torch.tensor(wdm, dtype=torch.float32, device=dev)
        # per-element multipliers for the CPU path
        if not self.gpu:
            self.lr_vec = torch.zeros(self.numel, dtype=torch.float32)
            self.wd_vec = torch.zeros(self.numel, dtype=torch.float32)
            self.mask = torch.zeros(self.numel, dtype=torch.bool)
            for p, o, l, w in zip(self.params, self.offsets, lrm, wdm):
                n = p.data.numel()
                self.lr_vec[o:o + n] = l
                self.wd_vec[o:o + n] = w
                self.mask[o:o + n] = True

    def zero_grad(self, lazy: bool = False):
        """Clear the flat gradient buffer.  ``lazy``: leave the slices of
        params whose gradient producer overwrites them on its first write
        (autograd.OVERWRITE_FIRST) -- one launch zeroes the rest; the caller
        then runs :meth:`fix_unwritten` after the backward."""
        ow = [i for i, p in enumerate(self.params) if p in autograd.OVERWRITE_FIRST] if lazy else []
        key = tuple(ow)
        if ow and self.gpu and getattr(self, "_zr_key", None) != key and N.lib().rt.is_capturing(N.stream()):
            ow = []  # (no host->device table upload inside a graph capture: clear everything)
        if not ow or not self.gpu:
            G.zero_(self.g)
        else:
            if getattr(self, "_zr_key", None) != key:
                # every table ever built stays alive (they are a few ints): a
                # HIP graph captured with an older key keeps zeroing from its
                # own table, never from a block the pool has handed out again
                tables = self.__dict__.setdefault("_zr_tables", {})
                if key not in tables:
                    skip = {self.offsets[i]: self.offsets[i] + self.params[i].data.numel() for i in ow}
                    ranges, cur = [], 0
                    for o in sorted(skip):
                        if o > cur:
                            ranges += [cur, o - cur]
                        cur = skip[o]
                    if cur < self.numel:
                        ranges += [cur, self.numel - cur]
                    t = memory.empty((len(ranges),), dtype=torch.int64, device=self.g.device)
                    G.copy_(t, torch.tensor(ranges, dtype=torch.int64))
                    tables[key] = t
                self._zr = tables[key]
                self._zr_key = key
            if self._zr.numel():
                N.lib().zero_ranges(self.g.data_ptr(), self._zr.data_ptr(), self._zr.numel() // 2, N.stream())
        autograd.GRAD_EPOCH[0] += 1

    def fix_unwritten(self):
        """Zero the gradients a lazy :meth:`zero_grad` left alone that this
        epoch's backward did not write (e.g. a branch that did not run)."""
        for p in self.params:
            if (p in autograd.OVERWRITE_FIRST
                    and autograd._WGRAD_EPOCH.get(id(p)) != autograd.GRAD_EPOCH[0]):
                G.zero_(p.grad_view)

    def sync_low(self):
        if self.low is not None:
            G.copy_(self.low, self.w)

    def param_range(self, i: int):
        return self.offsets[i], self.params[i].data.numel()

    def state_dict(self) -> Dict[str, torch.Tensor]:
        d = {"w": self.w}
        if self.s1 is not None:
            d["s1"] = self.s1
        if self.s2 is not None:
            d["s2"] = self.s2
        return d

    def slot_views(self, flat: torch.Tensor) -> List[torch.Tensor]:
        """Per-parameter views of a flat buffer of this store's layout, in
        each parameter's LOGICAL shape (conv weights KCRS whatever the flat
        memory order is)."""
        return [self._view(flat, o, p.data.shape) for p, o in zip(self.params, self.offsets)]

    def export_slot(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Device-independent form of an optimiser slot: one logical-layout
        tensor per parameter (``"<index>"`` in store order).  A flat dump is
        NOT portable: the GPU store keeps conv weights KRSC, the CPU store
        KCRS, with the same numel -- a raw copy would scramble them."""
        return {str(i): v.detach().contiguous().cpu() for i, v in enumerate(self.slot_views(flat))}

    def import_slot(self, flat: torch.Tensor, parts: Dict[str, torch.Tensor]) -> None:
        views = self.slot_views(flat)
        if len(parts) != len(views):
            raise ValueError(f"optimizer slot has {len(parts)} tensors, store has {len(views)} parameters")
        for i, v in enumerate(views):
            t = torch.as_tensor(parts[str(i)])
            if tuple(t.shape) != tuple(v.shape):
                raise ValueError(f"optimizer slot tensor {i}: shape {tuple(t.shape)} != parameter {tuple(v.shape)}")
            v.copy_(t.to(device=v.device, dtype=v.dtype))


# ---------------------------------------------------------------------------
_KIND = {"sgd": 0, "nesterov_ref": 1, "adagrad": 2, "rmsprop": 3, "adadelta": 4, "adam": 5, "sgd_ref": 6}


class Optimizer:
    """Base optimiser (SINGA opt API).  ``opt(loss)`` = backward + update."""

    kind = "sgd"
    state_slots = 1

    def __init__(self, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, beta1=0.9,
                 beta2=0.999, eps=1e-8, rho=0.9, adamw=False, dtype=torch.float32):
        self.lr = _sched(lr)
        self.momentum, self.dampening, self.weight_decay, self.nesterov = momentum, dampening, weight_decay, nesterov
        self.beta1, self.beta2, self.eps, self.rho, self.adamw = beta1, beta2, eps, rho, adamw
        self.step_counter = 0
        self.store: Optional[ParamStore] = None
        self.mixed_bf16 = False
        self.grad_scale = 1.0
        self._hp_dev = None
        self._hp_host = None
        self.graph_mode = False
        self._per_param: Dict[int, Dict[str, torch.Tensor]] = {}

    # -- configuration -----------------------------------------------------
    def attach(self, params: Sequence[Tensor], mixed_bf16: bool = False,
               channels_last: Optional[bool] = None) -> ParamStore:
        self.mixed_bf16 = mixed_bf16
        self.store = ParamStore(params, mixed_bf16=mixed_bf16, state_slots=2 if self.kind in (
            "adam", "adadelta") else 1, channels_last=channels_last)
        dev = self.store.device
        self._hp_dev = G.zeros((4,), torch.float32, dev)
        self._hp_host = torch.zeros(4, dtype=torch.float32, pin_memory=dev.type == "cuda")
        self.prepare_step()
        return self.store

    def current_lr(self) -> float:
        return float(self.lr(self.step_counter))

    def prepare_step(self) -> None:
        """Write (lr, t) for the NEXT update into the device hp buffer (call
        outside graph capture; the captured update kernel reads it)."""
        if self._hp_dev is None:
            return
        # two scalar fill kernels: the values travel as kernel arguments, so
        # the host can run ahead of the GPU without racing a pinned staging
        # buffer that an earlier, still-queued async copy would read later
        G.fill_(self._hp_dev[0], self.current_lr())
        G.fill_(self._hp_dev[1], float(self.step_counter + 1))

    # -- SINGA API -----------------------------------------------------------
    def __call__(self, loss: Tensor) -> None:
        self.backward_and_update(loss)

    def call(self, loss: Tensor) -> None:
        for p, g in autograd.backward(loss):
            if self.store is None:
                self.apply(p.name, p, g)

    def backward_and_update(self, loss: Tensor) -> None:
        if self.store is None:
            self.call(loss)
            self.step()
            return
        self.store.zero_grad(lazy=LAZY_ZERO)
        for _ in autograd.backward(loss):
            pass
        self.store.fix_unwritten()
        self.update()
        self.step()

    def step(self) -> None:
        self.step_counter += 1
        if not self.graph_mode:
            self.prepare_step()

    def update(self, grad_scale: Optional[float] = None, g: Optional[torch.Tensor] = None) -> None:
        """One fused update of every parameter in the store (``g``: another
        flat gradient buffer of the store's layout, e.g. an executor thread's)."""
        st = self.store
        gs = self.grad_scale if grad_scale is None else grad_scale
        g = st.g if g is None else g
        assert g.numel() == st.numel and g.dtype == torch.float32
        if st.gpu:
            N.lib().opt_update(_KIND[self.kind], st.w.data_ptr(), g.data_ptr(), N.ptr(st.s1), N.ptr(st.s2),
                               N.ptr(st.low), st.cstart.data_ptr(), st.clen.data_ptr(), st.cseg.data_ptr(),
                               st.seg_lr.data_ptr(), st.seg_wd.data_ptr(), self._hp_dev.data_ptr(), st.nchunks,
                               self.momentum, self.dampening, self.weight_decay, gs, self.beta1, self.beta2, self.eps,
                               self.rho, int(self.nesterov), int(self.adamw), N.stream())
            return
        if _native_cpu() is not None and st.w.is_contiguous() and g.is_contiguous():
            # CppCPU: the C++ updater of the host runtime (csrc/runtime/updater.cc)
            C = _native_cpu()
            C.opt_update(C.updater_kind(self.kind), st.w.numpy(), g.numpy(),
                         st.s1.numpy() if st.s1 is not None else None,
                         st.s2.numpy() if st.s2 is not None else None,
                         self.current_lr(), self.weight_decay, gs, float(self.step_counter + 1),
                         momentum=self.momentum, dampening=self.dampening, beta1=self.beta1, beta2=self.beta2,
                         eps=self.eps, rho=self.rho, nesterov=bool(self.nesterov), adamw=bool(self.adamw),
                         lr_vec=st.lr_vec.numpy(), wd_vec=st.wd_vec.numpy(), mask=st.mask.numpy().view(np.uint8))
        else:
            self._cpu_update(st.w, g, st.s1, st.s2, st.lr_vec * self.current_lr(), st.wd_vec * self.weight_decay,
                             float(self.step_counter + 1), gs, st.mask)
        if st.low is not None:
            st.low.copy_(st.w)

    def update_range(self, i0: int, i1: int, grad_scale: Optional[float] = None) -> None:
        """The fused update of store parameters [i0, i1) only (a contiguous
        range of the flat buffers): the per-parameter schedule, where a
        parameter is updated as soon as its gradient is final in the backward
        (reference Worker::Update per param, src/worker/worker.cc:290-292)."""
        st = self.store
        if i0 >= i1:
            return
        gs = self.grad_scale if grad_scale is None else grad_scale
        o0 = st.offsets[i0]
        o1 = st.offsets[i1] if i1 < len(st.params) else st.numel
        if st.gpu:
            c0, c1 = st.chunk_lo[i0], st.chunk_lo[i1] if i1 < len(st.params) else st.nchunks
            N.lib().opt_update(_KIND[self.kind], st.w.data_ptr(), st.g.data_ptr(), N.ptr(st.s1), N.ptr(st.s2),
                               N.ptr(st.low), st.cstart[c0:].data_ptr(), st.clen[c0:].data_ptr(),
                               st.cseg[c0:].data_ptr(), st.seg_lr.data_ptr(), st.seg_wd.data_ptr(),
                               self._hp_dev.data_ptr(), c1 - c0, self.momentum, self.dampening, self.weight_decay, gs,
                               self.beta1, self.beta2, self.eps, self.rho, int(self.nesterov), int(self.adamw),
                               N.stream())
            return
        sl = slice(o0, o1)
        w, g = st.w[sl], st.g[sl]
        s1 = st.s1[sl] if st.s1 is not None else None
        s2 = st.s2[sl] if st.s2 is not None else None
        if _native_cpu() is not None and st.w.is_contiguous() and st.g.is_contiguous():
            C = _native_cpu()
            C.opt_update(C.updater_kind(self.kind), w.numpy(), g.numpy(), s1.numpy() if s1 is not None else None,
                         s2.numpy() if s2 is not None else None, self.current_lr(), self.weight_decay, gs,
                         float(self.step_counter + 1), momentum=self.momentum, dampening=self.dampening,
                         beta1=self.beta1, beta2=self.beta2, eps=self.eps, rho=self.rho,
                         nesterov=bool(self.nesterov), adamw=bool(self.adamw), lr_vec=st.lr_vec[sl].numpy(),
                         wd_vec=st.wd_vec[sl].numpy(), mask=st.mask[sl].numpy().view(np.uint8))
        else:
            self._cpu_update(w, g, s1, s2, st.lr_vec[sl] * self.current_lr(), st.wd_vec[sl] * self.weight_decay,
                             float(self.step_counter + 1), gs, st.mask[sl])
        if st.low is not None:
            st.low[sl].copy_(w)

    # reference math on flat fp32 buffers (CPU)
    def _cpu_update(self, w, g, s1, s2, lr, wd, t, gs, mask=None):
        k = self.kind
        gv = g * gs
        if not (k == "adam" and self.adamw):
            gv = gv + wd * w
        if k == "sgd":
            if self.momentum != 0:
                s1.mul_(self.momentum).add_((1 - self.dampening) * gv)
                gv = gv + self.momentum * s1 if self.nesterov else s1
            upd = lr * gv
        elif k == "sgd_ref":
            if self.momentum > 0:
                s1.mul_(self.momentum).add_(lr * gv)
                upd = s1.clone()
            else:
                upd = lr * gv
        elif k == "nesterov_ref":
            h0 = s1.clone()
            s1.mul_(self.momentum).add_(lr * gv)
            upd = (1 + self.momentum) * s1 - self.momentum * h0
        elif k == "adagrad":
            s1.add_(gv * gv)
            upd = lr * gv / torch.sqrt(s1 + self.eps)
        elif k == "rmsprop":
            s1.mul_(self.rho).add_((1 - self.rho) * gv * gv)
            upd = lr * gv / torch.sqrt(s1 + self.eps)
        elif k == "adadelta":
            s1.mul_(self.rho).add_((1 - self.rho) * gv * gv)
            d = gv * torch.sqrt(s2 + self.eps) / torch.sqrt(s1 + self.eps)
            s2.mul_(self.rho).add_((1 - self.rho) * d * d)
            upd = lr * d
        elif k == "adam":
            s1.mul_(self.beta1).add_((1 - self.beta1) * gv)
            s2.mul_(self.beta2).add_((1 - self.beta2) * gv * gv)
            mh = s1 / (1 - self.beta1 ** t)
            vh = s2 / (1 - self.beta2 ** t)
            upd = lr * (mh / (torch.sqrt(vh) + self.eps) + (wd * w if self.adamw else 0.0))
        else:
            raise ValueError(k)
        if mask is not None:
            upd = torch.where(mask, upd, torch.zeros_like(upd))
        w.sub_(upd)

    def apply(self, param_name: str, param_value: Tensor, param_grad: Tensor) -> None:
        """Per-parameter update (used before/without a ParamStore)."""
        w = param_value.data
        g = param_grad.data.reshape(w.shape).float()
        st = self._per_param.setdefault(id(param_value), {})
        if "s1" not in st:
            st["s1"] = torch.zeros_like(w, dtype=torch.float32)
            st["s2"] = torch.zeros_like(w, dtype=torch.float32)
        meta = param_value.param_meta or {}
        lr = self.current_lr() * meta.get("lr_mult", 1.0)
        wd = self.weight_decay * meta.get("wd_mult", 1.0)
        wf = w.float()
        self._cpu_update(wf, g, st["s1"], st["s2"], lr, wd, float(self.step_counter + 1), self.grad_scale)
        if wf is not w:
            w.copy_(wf)
        if param_value.low is not None:
            param_value.low.copy_(w)

    # -- checkpoint ----------------------------------------------------------
    def get_states(self) -> Dict[str, object]:
        d: Dict[str, object] = {"step_counter": self.step_counter, "kind": self.kind, "slot_layout": "logical"}
        if self.store is not None:
            for k in ("s1", "s2"):
                flat = getattr(self.store, k)
                if flat is not None:
                    for i, t in self.store.export_slot(flat).items():
                        d[f"{k}/{i}"] = t
        return d

    def set_states(self, states: Dict[str, object]) -> None:
        self.step_counter = int(states.get("step_counter", 0))
        if self.store is not None:
            for k in ("s1", "s2"):
                flat = getattr(self.store, k)
                if flat is None:
                    continue
                parts = {key[len(k) + 1:]: v for key, v in states.items() if key.startswith(k + "/")}
                if parts:
                    self.store.import_slot(flat, parts)
                elif k in states:
                    # legacy flat dump (layout of the saving device unknown):
                    # only safe when saved and loaded on the same kind of device
                    import warnings

                    warnings.warn(f"optimizer state '{k}' is a legacy flat buffer; restoring it assumes the "
                                  "checkpoint was written on the same device type")
                    flat.copy_(torch.as_tensor(states[k]))
        self.prepare_step()


class SGD(Optimizer):
    kind = "sgd"

    def __init__(self, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, dtype=torch.float32):
        super().__init__(lr, momentum, dampening, weight_decay, nesterov, dtype=dtype)


class RefSGD(Optimizer):
    """The reference's SGDUpdater: h = m*h + lr*g; w -= h (src/utils/updater.cc:62-80)."""
    kind = "sgd_ref"

    def __init__(self, lr=0.1, momentum=0.0, weight_decay=0.0):
        super().__init__(lr, momentum, 0.0, weight_decay)


class Nesterov(Optimizer):
    """Reference NesterovUpdater (src/utils/updater.cc:82-105), momentum set."""
    kind = "nesterov_ref"

    def __init__(self, lr=0.1, momentum=0.9, weight_decay=0.0):
        super().__init__(lr, momentum, 0.0, weight_decay)


class AdaGrad(Optimizer):
    kind = "adagrad"

    def __init__(self, lr=0.01, epsilon=1e-8, weight_decay=0.0):
        super().__init__(lr, weight_decay=weight_decay, eps=epsilon)


class RMSProp(Optimizer):
    kind = "rmsprop"

    def __init__(self, lr=0.01, rho=0.9, epsilon=1e-8, weight_decay=0.0):
        super().__init__(lr, weight_decay=weight_decay, eps=epsilon, rho=rho)


class AdaDelta(Optimizer):
    kind = "adadelta"
    state_slots = 2

    def __init__(self, lr=1.0, rho=0.95, epsilon=1e-6, weight_decay=0.0):
        super().__init__(lr, weight_decay=weight_decay, eps=epsilon, rho=rho)


class Adam(Optimizer):
    kind = "adam"
    state_slots = 2

    def __init__(self, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-8, weight_decay=0.0, adamw=False):
        super().__init__(lr, weight_decay=weight_decay, beta1=beta_1, beta2=beta_2, eps=epsilon, adamw=adamw)


class AdamW(Adam):
    def __init__(self, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-8, weight_decay=0.01):
        super().__init__(lr, beta_1, beta_2, epsilon, weight_decay, adamw=True)


def DistOpt(*args, **kwargs):
    """Alias to :class:`singa_amd.parallel.distopt.DistOpt` (SINGA path)."""
    from .parallel.distopt import DistOpt as _D

    return _D(*args, **kwargs)
