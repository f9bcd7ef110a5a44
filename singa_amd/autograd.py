"""``singa_amd.autograd`` -- SINGA's operator-tape autograd.

Operators record their inputs when ``autograd.training`` is True; the
:func:`backward` generator walks the tape in dependency order and yields
``(param, grad)`` pairs the moment a parameter's gradient is complete -- the
hook that lets :class:`singa_amd.opt.DistOpt` launch bucketed RCCL
all-reduces while the rest of the backward pass is still running (the
reference interleaves ``UpdateParam`` with ``ComputeGradient`` in the same way,
src/worker/worker.cc:270-302).

Hot operators (convolution, linear, batch-norm(+ReLU, +residual), pooling,
activations, softmax-cross-entropy, dropout, LRN, layer-norm) call the
gfx950 kernels through :mod:`singa_amd.ops.functional`.  Parameters that live
in a flat :class:`singa_amd.opt.ParamStore` carry an fp32 ``grad_view``; the
conv/linear/BN backward kernels accumulate straight into it (no per-param
gradient tensors, one fused optimiser launch afterwards).  Non-hot "glue"
operators (shape manipulation, ONNX odds and ends) are :class:`Fn` operators
whose forward and backward are explicit functions over native glue kernels
(views: their inverse view) -- the tape is the only autograd engine.
"""
from __future__ import annotations

import builtins as _b
import math
import os
import sys
import threading
import types
import heapq
import weakref
from collections import Counter, deque
from typing import Callable, Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import memory as _mem
from . import tensor as _tensor
from .ops import functional as F
from .ops import glue as G
from .ops import native as N
from .tensor import Tensor

# ``autograd.training`` is per THREAD (a property of this module's class over
# thread-local storage): ranks driven as threads (parallel.fake) and hogwild
# replicas each toggle their own flag -- a module global let one thread's
# compile() (tape-free forward) switch off another thread's tape mid-step.
_TLS = threading.local()


def _training() -> bool:
    return getattr(_TLS, "training", False)


class _AutogradModule(types.ModuleType):
    @property
    def training(self) -> bool:
        return getattr(_TLS, "training", False)

    @training.setter
    def training(self, v) -> None:
        _TLS.training = bool(v)


sys.modules[__name__].__class__ = _AutogradModule

ACCUMULATED = object()  # backward() returned: grad already added to the param's grad_view
# ParamStore.zero_grad() bumps GRAD_EPOCH; a conv records the epoch in which it
# last added to its weight gradient (the identity-sum BN backward needs that
# gradient to hold this backward's contribution only)
GRAD_EPOCH = [0]
_WGRAD_EPOCH: dict = {}
# params whose gradient a Linear writes (beta = 0, no zeroed buffer needed) on
# its first contribution in an epoch; ParamStore.zero_grad(lazy=True) leaves
# their slices alone and fix_unwritten() zeroes any that a step did not reach
OVERWRITE_FIRST = weakref.WeakSet()  # the param Tensors themselves (ids get reused)
# uses of each param (id) in the current backward (its producers may only
# overwrite the gradient when they are the sole user)
PARAM_USES: dict = {}
# backward() returned: the input gradient was added IN PLACE into the partial
# gradient the engine offered through ``op.acc_into`` (see backward())
ACC_INPLACE = object()
INPLACE_ACC = os.environ.get("SINGA_AMD_INPLACE_ACC", "1") != "0"  # (A/B switch)


class AccReplace:
    """backward() returned: the input gradient was summed with the partial
    gradient the engine offered through ``op.acc_into`` into the NEW tensor
    ``t``, which replaces that partial gradient (a dgrad epilogue that adds
    the other consumers' gradient from its own buffer)."""

    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t  # engine switch (tests A/B the in-place accumulation against separate adds)


def _as_tuple(x):
    return x if isinstance(x, tuple) else (x,)


_SEQ = [0]
_TRACE: list = []  # stack of op-record lists (sonnx.to_onnx tracing)


def _next_seq() -> int:
    _SEQ[0] += 1
    return _SEQ[0]


class Operator:
    """Base operator.  Subclasses implement ``forward(*raw)`` and
    ``backward(*raw_dys)`` on ``torch.Tensor`` storage."""

    op_count = 0

    def __init__(self, name: Optional[str] = None):
        if name is None:
            name = f"{type(self).__name__}#{Operator.op_count}"
            Operator.op_count += 1
        self.name = name
        self.src: List = []
        self.params: List[Optional[Tensor]] = []
        self.requires_grad = False

    def __call__(self, *xs):
        return self._do_forward(*xs)

    def _do_forward(self, *xs):
        xs = tuple(x if isinstance(x, Tensor) else Tensor(data=x, requires_grad=False) for x in xs)
        self.requires_grad = _training() and any(x.requires_grad for x in xs)
        if self.requires_grad:
            self.src = [(x.creator, x.stores_grad) for x in xs]
            self.src_idx = [x.creator._yid.get(id(x), 0) if x.creator is not None else 0 for x in xs]
            self.params = [x if x.stores_grad else None for x in xs]
            self.input_requires = [x.requires_grad for x in xs]
            self.src_dt = [x.dtype for x in xs]
        ys = _as_tuple(self.forward(*[x.data for x in xs]))
        dev = xs[0].device
        outs = tuple(
            Tensor(device=dev, data=y, requires_grad=self.requires_grad,
                   creator=self if self.requires_grad else None) for y in ys)
        if self.requires_grad:
            self.n_out = len(outs)
            self._yid = {id(o): i for i, o in enumerate(outs)}
            self._seq = _next_seq()
        if _TRACE:  # sonnx export: record (op, inputs, outputs)
            _TRACE[-1].append((self, xs, outs))
        return outs[0] if len(outs) == 1 else outs

    def grad_target(self, i: int) -> Optional[torch.Tensor]:
        """fp32 flat-buffer gradient view of input i if it is a stored param."""
        if i < len(self.params) and self.params[i] is not None:
            return self.params[i].grad_view
        return None

    def needs_grad(self, i: int) -> bool:
        return getattr(self, "input_requires", [True] * (i + 1))[i]

    def forward(self, *xs):
        raise NotImplementedError

    def backward(self, *dys):
        raise NotImplementedError

    def get_params(self):
        return {}


class Dummy(Operator):
    """Leaf marker (SINGA compatibility)."""

    def __init__(self, tensor: Tensor, name=None):
        super().__init__(name)
        self.tensor = tensor


def infer_dependency(op: Operator) -> Dict[Operator, int]:
    """Number of consumers of each operator reachable from ``op``."""
    deps: Counter = Counter()
    seen = {op}
    q = deque([op])
    while q:
        cur = q.popleft()
        for src_op, _ in cur.src:
            if src_op is None:
                continue
            deps[src_op] += 1
            if src_op not in seen:
                seen.add(src_op)
                q.append(src_op)
    return deps


def _param_uses(op: Operator) -> Counter:
    uses: Counter = Counter()
    seen = {op}
    q = deque([op])
    while q:
        cur = q.popleft()
        for p in cur.params:
            if p is not None:
                uses[id(p)] += 1
        for src_op, _ in cur.src:
            if src_op is not None and src_op not in seen:
                seen.add(src_op)
                q.append(src_op)
    return uses


def _accum(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if isinstance(a, F.LAZY_GRADS):  # a lazy gradient meets another contribution
        a = a.materialize()
    if isinstance(b, F.LAZY_GRADS):
        b = b.materialize()
    if a.shape != b.shape:
        b = G.reshape(b, a.shape)
    if a.dtype != b.dtype:
        b = G.to(b, a.dtype)
    if a.stride() == b.stride() and a.is_cuda and (a.is_contiguous() or N.is_cl(a)):
        return F.add_act(a, b)
    return G.binary("add", a, b)


def is_unit(dy) -> bool:
    """True if dy is the implicit d(loss)/d(loss) = 1 seed."""
    return dy is None or getattr(dy, "_sg_unit", False)


def backward(y, dy=None) -> Iterator[Tuple[Tensor, Tensor]]:
    """Generator of (param, grad) in the order gradients complete.

    ``y`` may be one tensor or a list of roots (with a matching list ``dy``;
    ``None`` seeds a loss with ones).  Ready operators run in decreasing
    forward order (a max-heap on the forward sequence number): gradients
    complete from the last layer backwards, which is what bucketed
    all-reduce overlap wants, and it gives every process the same global
    order, which the cross-process bridge operators rely on (see
    :mod:`singa_amd.runtime.neuralnet`)."""
    roots = list(y) if isinstance(y, (list, tuple)) else [y]
    dys = list(dy) if isinstance(dy, (list, tuple)) else [dy] * len(roots)
    heap: List = []
    pending: Dict[Operator, list] = {}
    puses: Counter = Counter()
    for r, d in zip(roots, dys):
        if r is None or r.creator is None:
            continue
        op0 = r.creator
        if op0 not in pending:
            pending[op0] = [None] * op0.n_out
        if d is None:
            g0 = G.full(r.data.shape, 1.0, r.data.dtype, r.data.device)
            g0._sg_unit = True
        else:
            g0 = d.data if isinstance(d, Tensor) else d
        j = op0._yid.get(id(r), 0)
        pending[op0][j] = _accum(pending[op0][j], g0)
    if not pending:
        return
    # dependency counts / param uses over the union of the root subgraphs
    deps = Counter()
    seen = set(pending)
    q = deque(pending)
    while q:
        cur = q.popleft()
        for p in cur.params:
            if p is not None:
                puses[id(p)] += 1
        for src_op, _ in cur.src:
            if src_op is None:
                continue
            deps[src_op] += 1
            if src_op not in seen:
                seen.add(src_op)
                q.append(src_op)
    for op_ in seen:  # consumers of each op's output in this backward (fusion decisions look ahead with it)
        op_._consumers = deps[op_]
    PARAM_USES.clear()
    PARAM_USES.update(puses)
    if OVERWRITE_FIRST:
        # a lazily-zeroed gradient slice with several users this time: clear
        # it now and let zero_grad cover it again
        for op_ in seen:
            for p in op_.params:
                # (only a Linear overwrites its weight gradient on its first
                # write: any other sole user would add into the stale slice)
                if p is not None and p in OVERWRITE_FIRST and (puses[id(p)] > 1 or not isinstance(op_, Linear)):
                    OVERWRITE_FIRST.discard(p)
                    if p.grad_view is not None and _WGRAD_EPOCH.get(id(p)) != GRAD_EPOCH[0]:
                        G.zero_(p.grad_view)
    # every conv weight this backward's data gradients need, transposed K-major in one launch
    convs = sorted((o for o in seen if isinstance(o, Conv2d) and getattr(o, "w", None) is not None and o.group == 1
                    and o.dilation == (1, 1) and o.needs_grad(0)), key=lambda o: getattr(o, "_seq", 0))
    if len(convs) > 1 and N.available() and convs[0].w.is_cuda:
        pre = F.pretranspose_conv_weights([(id(o), o.w) for o in convs])
        for o in convs:
            o.wt_pre = pre.get(id(o))
    for op0 in pending:
        if deps[op0] == 0:
            heapq.heappush(heap, (-getattr(op0, "_seq", 0), id(op0), op0))
    pgrad: Dict[int, object] = {}
    # ids of pending partial gradients the engine exclusively owns (fresh
    # buffers produced by one backward, or sums it made): an operator that
    # declares ``accepts_acc`` may add its input gradient into such a buffer
    # in place (e.g. the conv dgrad epilogue with beta=1) instead of
    # returning a new tensor for a separate add pass
    owned: set = set()
    while heap:
        op = heapq.heappop(heap)[2]
        dys_ = pending.pop(op)
        for d in dys_:
            if d is not None:
                owned.discard(id(d))
        # a lazy residual gradient nobody absorbed reaches its producer: make it a tensor
        dys_ = [d.materialize() if isinstance(d, F.LAZY_GRADS) else d for d in dys_]
        if all(d is None for d in dys_) and not getattr(op, "always_run", False):
            dxs = (None,) * len(op.src)
        else:
            if INPLACE_ACC and getattr(op, "accepts_acc", False):
                acc, last = {}, {}
                for i, (src_op, _) in enumerate(op.src):
                    if src_op is not None and op.params[i] is None and src_op in pending:
                        cur = pending[src_op][op.src_idx[i]]
                        if cur is not None and id(cur) in owned:
                            acc[i] = cur
                            # this op's contribution completes src_op's gradient
                            last[i] = deps[src_op] == 1 and src_op.n_out == 1
                op.acc_into = acc
                op.acc_last = last
            if getattr(op, "wants_sole", False):
                # input i's producer gets its whole gradient from this op alone
                op.sole = {i: src_op is not None and deps[src_op] == 1 and src_op not in pending
                           and src_op.n_out == 1 for i, (src_op, _) in enumerate(op.src)}
            dxs = _as_tuple(op.backward(*dys_))
            op.acc_into = op.acc_last = None
        if len(dxs) != len(op.src):
            raise RuntimeError(f"{op.name}: backward returned {len(dxs)} grads for {len(op.src)} inputs")
        for i, ((src_op, stores), dx) in enumerate(zip(op.src, dxs)):
            p = op.params[i]
            if p is not None:
                key = id(p)
                if dx is ACCUMULATED:
                    pgrad.setdefault(key, ACCUMULATED)
                elif dx is not None:
                    prev = pgrad.get(key)
                    if p.grad_view is not None:
                        G.binary("add", p.grad_view, G.reshape(dx, p.grad_view.shape), out=p.grad_view)
                        pgrad[key] = ACCUMULATED
                    else:
                        pgrad[key] = _accum(prev, dx)
                puses[key] -= 1
                if puses[key] == 0:
                    g = pgrad.pop(key, None)
                    if g is ACCUMULATED:
                        g = p.grad_view
                    if g is not None:
                        yield p, Tensor(device=p.device, data=g, requires_grad=False)
                continue
            if src_op is None:
                continue
            if isinstance(dx, AccReplace):
                j = op.src_idx[i]
                prev = pending[src_op][j]
                if prev is not None:
                    owned.discard(id(prev))
                pending[src_op][j] = dx.t
                owned.add(id(dx.t))
                deps[src_op] -= 1
                if deps[src_op] == 0:
                    heapq.heappush(heap, (-getattr(src_op, "_seq", 0), id(src_op), src_op))
                continue
            if dx is ACCUMULATED or dx is ACC_INPLACE:
                dx = None  # (ACC_INPLACE: already summed into pending[src_op])
            elif dx is not None and dx.dtype != op.src_dt[i] and dx.is_floating_point():
                dx = G.to(dx, op.src_dt[i])  # mixed-precision edge: grads take the producer's dtype
            if src_op not in pending:
                pending[src_op] = [None] * src_op.n_out
            j = op.src_idx[i]
            prev = pending[src_op][j]
            new = _accum(prev, dx)
            if new is not prev:
                if prev is not None:
                    owned.discard(id(prev))
                    if dx is not None:  # a sum the engine just allocated
                        owned.add(id(new))
                elif getattr(new, "_sg_fresh", False) and len([d for d in dxs if d is new]) == 1:
                    owned.add(id(new))
            pending[src_op][j] = new
            deps[src_op] -= 1
            if deps[src_op] == 0:
                heapq.heappush(heap, (-getattr(src_op, "_seq", 0), id(src_op), src_op))


def gradients(y: Tensor, dy: Optional[Tensor] = None) -> Dict[Tensor, Tensor]:
    return {p: g for p, g in backward(y, dy)}


# ===========================================================================
# hot operators (native kernels on GPU)
# ===========================================================================
class _Unary(Operator):
    kind = "identity"
    needs = "x"  # which saved tensor the backward needs: "x", "y" or "xy"

    def __init__(self, alpha: float = 0.0, name=None):
        super().__init__(name)
        self.alpha = alpha

    def forward(self, x):
        y = F.unary(self.kind, x, self.alpha)
        if self.requires_grad:
            self.x = x if "x" in self.needs else None
            self.y = y if "y" in self.needs else None
        return y

    def backward(self, dy):
        if getattr(self, "bwd_done", False):
            # the consuming Linear's data-gradient GEMM applied this
            # activation's derivative in its epilogue: dy is already dx
            self.bwd_done = False
            self.x = self.y = None
            return dy
        dx = F.unary_bwd(self.kind, self.x, self.y, dy, self.alpha)
        self.x = self.y = None
        return dx


class ReLU(_Unary):
    kind = "relu"
    needs = "y"

    def backward(self, dy):
        if getattr(self, "bwd_done", False):  # (applied by the consuming Linear's dgrad epilogue)
            self.bwd_done = False
            self.y = None
            return dy
        dx = F.relu_bwd_from_y(self.y, dy)
        self.y = None
        return dx


class Sigmoid(_Unary):
    kind, needs = "sigmoid", "y"


class Tanh(_Unary):
    kind, needs = "tanh", "y"


class STanh(_Unary):
    """LeCun scaled tanh 1.7159*tanh(2/3 x) -- the reference's kTanh layer
    (include/mshadow/cxxnet_op.h:77-87)."""
    kind, needs = "stanh", "y"


class Gelu(_Unary):
    kind, needs = "gelu", "x"


class SoftPlus(_Unary):
    kind, needs = "softplus", "x"


class Exp(_Unary):
    kind, needs = "exp", "y"


class Log(_Unary):
    kind, needs = "log", "x"


class Abs(_Unary):
    kind, needs = "abs", "x"


class Sqrt(_Unary):
    kind, needs = "sqrt", "y"


class Reciprocal(_Unary):
    kind, needs = "reciprocal", "y"


class Negative(_Unary):
    kind, needs = "neg", ""


class Sign(_Unary):
    kind, needs = "sign", ""


class Square(_Unary):
    kind, needs = "square", "x"


class LeakyRelu(_Unary):
    kind, needs = "leakyrelu", "x"

    def __init__(self, a: float = 0.01, name=None):
        super().__init__(a, name)


class Elu(_Unary):
    kind, needs = "elu", "xy"

    def __init__(self, alpha: float = 1.0, name=None):
        super().__init__(alpha, name)


class SeLU(_Unary):
    kind, needs = "selu", "xy"

    def __init__(self, alpha: float = 1.67326, gamma: float = 1.0507, name=None):
        super().__init__(0.0, name)


class Identity(Operator):
    def forward(self, x):
        return x

    def backward(self, dy):
        return dy


def _unbroadcast(g: torch.Tensor, shape) -> torch.Tensor:
    return G.sum_to(g, shape)


class Add(Operator):
    def __init__(self, relu: bool = False, name=None):
        super().__init__(name)
        self.relu = relu

    def forward(self, a, b):
        if a.shape == b.shape and a.dtype == b.dtype and (a.stride() == b.stride()) and (
                a.is_contiguous() or N.is_cl(a)):
            y = F.add_act(a, b, relu=self.relu)
        else:
            y = G.binary("add", a, b)
            if self.relu:
                y = F.unary("relu", y)
        if self.requires_grad:
            self.sa, self.sb = a.shape, b.shape
            self.y = y if self.relu else None
        return y

    def backward(self, dy):
        if self.relu:
            dy = F.relu_bwd_from_y(self.y, dy)
            self.y = None
        return _unbroadcast(dy, self.sa), _unbroadcast(dy, self.sb)


class Sub(Operator):
    def forward(self, a, b):
        if self.requires_grad:
            self.sa, self.sb = a.shape, b.shape
        return G.binary("sub", a, b)

    def backward(self, dy):
        return _unbroadcast(dy, self.sa), _unbroadcast(F.unary("neg", dy), self.sb)


class Mul(Operator):
    def forward(self, a, b):
        if self.requires_grad:
            self.a, self.b = a, b
        return G.binary("mul", a, b)

    def backward(self, dy):
        a, b = self.a, self.b
        self.a = self.b = None
        da = _unbroadcast(G.binary("mul", dy, b, out_dtype=a.dtype), a.shape) if self.needs_grad(0) else None
        db = _unbroadcast(G.binary("mul", dy, a, out_dtype=b.dtype), b.shape) if self.needs_grad(1) else None
        return da, db


class Div(Operator):
    def forward(self, a, b):
        y = G.binary("div", a, b)
        if self.requires_grad:
            self.b, self.y = b, y
            self.sa = a.shape
        return y

    def backward(self, dy):
        b, y = self.b, self.y
        self.b = self.y = None
        da = G.binary("div", dy, b)  # d/da = dy / b ; d/db = -dy * y / b
        db = G.binary("mul", G.binary("div", dy, b), y, alpha=-1.0) if self.needs_grad(1) else None
        return _unbroadcast(da, self.sa), (_unbroadcast(db, b.shape) if db is not None else None)


class Pow(Operator):
    def forward(self, a, b):
        y = G.binary("pow", a, b)
        if self.requires_grad:
            self.a, self.b, self.y = a, b, y
        return y

    def backward(self, dy):
        a, b, y = self.a, self.b, self.y
        self.a = self.b = self.y = None
        # da = dy * b * a^(b-1) ; db = dy * y * log(a)
        da = G.binary("mul", G.binary("mul", dy, b), G.binary("pow", a, F.unary("adds", b, -1.0)))
        db = None
        if self.needs_grad(1):
            la = F.unary("log", G.clamp_affine(a, lo=1e-30))
            db = G.binary("mul", G.binary("mul", dy, y), la)
        return _unbroadcast(da, a.shape), (_unbroadcast(db, b.shape) if db is not None else None)


class Matmul(Operator):
    """Batched/2-D matrix product: bf16 operands on the MFMA kernel, fp32 on
    the exact-f32 MFMA kernel (functional.gemm); backward likewise."""

    def forward(self, a, b):
        if self.requires_grad:
            self.a, self.b = a, b
        return F.matmul(a, b, out_dtype=a.dtype)

    def backward(self, dy):
        a, b = self.a, self.b
        self.a = self.b = None
        dy = dy.contiguous()
        if a.dim() == 2 and b.dim() == 2:
            da = F.gemm_nt(dy, b, out_dtype=a.dtype) if self.needs_grad(0) else None
            db = None
            if self.needs_grad(1):
                tgt = self.grad_target(1)
                if tgt is not None:
                    F.gemm_tn_acc(a, dy, tgt)
                    db = ACCUMULATED
                else:
                    db = F.gemm(a, dy, ta=True, out_dtype=b.dtype)
            return da, db
        # batched: flatten leading dims (broadcast operands are reduced by _unbroadcast)
        lead = torch.broadcast_shapes(a.shape[:-2], b.shape[:-2])
        a3 = G.reshape(a.expand(*lead, *a.shape[-2:]), (-1, *a.shape[-2:]))
        b3 = G.reshape(b.expand(*lead, *b.shape[-2:]), (-1, *b.shape[-2:]))
        d3 = G.reshape(dy, (-1, *dy.shape[-2:]))
        da = db = None
        if self.needs_grad(0):
            da = _unbroadcast(F.gemm(d3, b3, tb=True, out_dtype=a.dtype).reshape(*lead, *a.shape[-2:]), a.shape)
        if self.needs_grad(1):
            db = _unbroadcast(F.gemm(a3, d3, ta=True, out_dtype=b.dtype).reshape(*lead, *b.shape[-2:]), b.shape)
        return da, db


class AddBias(Operator):
    """y = x + b broadcast along ``axis`` (SINGA AddBias: axis 0 adds a row)."""

    def __init__(self, axis: int = 0, name=None):
        super().__init__(name)
        self.axis = axis

    def forward(self, x, b):
        bb = G.to(b, x.dtype)
        return G.binary("add", x, bb.reshape(1, -1) if self.axis == 0 else bb.reshape(-1, 1))

    def backward(self, dy):
        db = G.reduce(dy, [0] if self.axis == 0 else [1], "sum", out_dtype=torch.float32)
        tgt = self.grad_target(1)
        if tgt is not None:
            G.binary("add", tgt, db.reshape(tgt.shape), out=tgt)
            return dy, ACCUMULATED
        return dy, db


class Linear(Operator):
    """y = act(x @ W (+ b)) with W [in, out] (SINGA / reference InnerProduct
    layout, src/worker/layer.cc:193-211; the optional activation is the
    reference's following kTanh / kReLU / kSigmoid layer, layer.cc:563-606,
    fused into the GEMM epilogue).  Mixed precision: when x is bf16 the bf16
    compute copy ``W.low`` is used and gradients accumulate in fp32.

    Backward: the activation derivative is applied to dy first -- unless the
    consumer of this op's output was a fused Linear that is its only
    consumer: that op's data-gradient GEMM already multiplied by act'(y) in
    its epilogue (``preact_done``), so the separate elementwise pass
    disappears from both directions."""

    wants_sole = True

    def __init__(self, has_bias=True, name=None, act: Optional[str] = None):
        super().__init__(name)
        self.has_bias = has_bias
        self.act = act
        self.y2 = None  # the activation output (y-form derivatives) ...
        self.z2 = None  # ... or its input (GELU), written by the forward epilogue
        self.preact_done = False
        self.db_done = False  # a consumer (DropAddLayerNorm) already summed the bias gradient into its view

    accepts_acc = True  # the data gradient can add into another consumer's pending gradient of x

    def forward(self, x, W, b=None):
        w = self._w_compute(x, W)
        lead = x.shape[:-1]
        x2 = G.reshape(x, (-1, x.shape[-1]))
        bias = G.to(b, torch.float32) if b is not None else None
        z = None
        if self.act in F.ACT_XFORM and self.requires_grad:
            z = _mem.empty((x2.shape[0], w.shape[-1]), dtype=x.dtype, device=x2.device)
        y = F.matmul(x2, w, out_dtype=x.dtype, bias=bias, act=self.act, act_aux=z)
        if self.requires_grad:
            self.x2, self.w = x2, w
            self.y2 = y if self.act is not None else None
            self.z2 = z
        return G.reshape(y, (*lead, y.shape[-1]))

    def _producer_act(self, x2):
        """The fused-activation Linear whose output is this op's input and
        whose gradient comes from this op alone, else None."""
        src = self.src[0][0] if self.src else None
        if not (isinstance(src, Linear) and src.act is not None and src.y2 is not None
                and (src.act not in F.ACT_XFORM or src.z2 is not None)
                and getattr(self, "sole", {}).get(0, False)):
            return None
        y = src.y2
        if y.data_ptr() != x2.data_ptr() or y.numel() != x2.numel():
            return None
        return src

    def _producer_unary(self):
        """The standalone activation op (GELU, tanh, ...) whose output is this
        op's input and whose gradient comes from this op alone: the data
        gradient GEMM can apply its derivative in the epilogue."""
        src = self.src[0][0] if self.src else None
        if not (ACT_GRAD_FUSE and isinstance(src, _Unary) and src.kind in F.GEMM_ACT and src.alpha == 0.0
                and (getattr(self, "sole", None) or {}).get(0, False)):
            return None
        t = src.x if src.kind in F.ACT_XFORM else src.y
        return src if t is not None else None

    def _w_compute(self, x, W):
        if x.dtype == W.dtype:
            return W
        p = self.params[1] if len(self.params) > 1 else None
        if p is not None and p.low is not None and x.dtype == torch.bfloat16:
            return p.low
        return G.to(W, x.dtype)

    def backward(self, dy):
        x2, w, y2, z2 = self.x2, self.w, self.y2, self.z2
        self.x2 = self.w = self.y2 = None
        dy2 = G.contiguous(G.reshape(dy, (-1, dy.shape[-1])))
        if self.act is not None and not self.preact_done:
            if self.act == "relu":
                dy2 = F.relu_bwd_from_y(y2, dy2)
            elif self.act in F.ACT_XFORM:
                dy2 = F.unary_bwd(self.act, z2, None, dy2)
            else:
                dy2 = F.unary_bwd(self.act, None, y2, dy2)
        self.preact_done = False
        self.z2 = None
        dx = None
        if self.needs_grad(0):
            prod = self._producer_act(x2)
            if prod is not None:
                t = prod.z2 if prod.act in F.ACT_XFORM else x2
                # the producer's bias gradient = column sums of this GEMM's
                # output (its pre-activation gradient): summed in the same epilogue
                # (bf16: the tuned kernel's epilogue; the fp32 generic GEMM sums
                # the bias gradient in the producer's weight-gradient GEMM for free)
                pb = prod.grad_target(2) if (prod.has_bias and BIAS_INPLACE and x2.dtype == torch.bfloat16) else None
                if not (pb is not None and pb.is_cuda and pb.dtype == torch.float32 and pb.is_contiguous()
                        and pb.numel() == x2.shape[-1]):
                    pb = None
                dx = F.gemm_nt(dy2, w, out_dtype=x2.dtype, act_grad=(prod.act, G.reshape(t, tuple(x2.shape))),
                               colsum_c=pb)
                prod.preact_done = True
                if pb is not None:
                    prod.db_done = True
            elif self._producer_unary() is not None and x2.is_cuda:
                un = self._producer_unary()
                t = un.x if un.kind in F.ACT_XFORM else un.y
                # the activation's producer: its bias gradient is the column
                # sum of this GEMM's output when the activation is its only consumer
                lin = un.src[0][0] if un.src else None
                pb = None
                if (isinstance(lin, Linear) and lin.has_bias and lin.act is None and BIAS_INPLACE
                        and getattr(lin, "_consumers", 0) == 1 and x2.dtype == torch.bfloat16):
                    pb = lin.grad_target(2)
                    if not (pb is not None and pb.is_cuda and pb.dtype == torch.float32 and pb.is_contiguous()
                            and pb.numel() == x2.shape[-1]):
                        pb = None
                dx = F.gemm_nt(dy2, w, out_dtype=x2.dtype, act_grad=(un.kind, G.reshape(t, tuple(x2.shape))),
                               colsum_c=pb)
                un.bwd_done = True
                if pb is not None:
                    lin.db_done = True
            else:
                # another consumer's gradient of x already pending (a residual
                # stream: the tail's ds): this data gradient adds into it in
                # its epilogue (beta 1) instead of a separate add pass
                acc = (getattr(self, "acc_into", None) or {}).get(0)
                if (acc is not None and acc.is_cuda and acc.dtype == x2.dtype and acc.is_contiguous()
                        and acc.numel() == x2.numel() and w.dtype == dy2.dtype == x2.dtype):
                    F.gemm(dy2, w, tb=True, out=G.reshape(acc, tuple(x2.shape)), beta=1.0)
                    dx = ACC_INPLACE
                else:
                    dx = F.gemm_nt(dy2, w, out_dtype=x2.dtype)
            if dx is not ACC_INPLACE:
                dx = G.reshape(dx, (*dy.shape[:-1], x2.shape[-1]))
        tgt = self.grad_target(1)
        tb = self.grad_target(2) if self.has_bias else None
        # dy's column sums already summed by its producer (DropAddLayerNorm's backward)
        cs_pre = getattr(dy, "_sg_colsum", None) if self.act is None else None
        db_done, self.db_done = self.db_done and tb is not None, False
        # the bias gradient (column sums of dy) rides along with the weight
        # gradient GEMM, which stages every dy tile anyway
        fuse_db = tb is not None and tgt is not None and tb.is_contiguous() and cs_pre is None and not db_done
        if tgt is not None:
            wid = id(self.params[1])
            # first (and sole) writer of this epoch's weight gradient: write
            # it (beta 0) instead of adding into a zeroed buffer
            empty = _WGRAD_EPOCH.get(wid) != GRAD_EPOCH[0]
            first = (empty and PARAM_USES.get(wid) == 1 and tgt.is_cuda and tgt.is_contiguous()
                     and x2.dtype == torch.float32 and dy2.dtype == torch.float32)
            if first:
                F.gemm(x2, dy2, ta=True, out=tgt, beta=0.0, colsum_b=tb if fuse_db else None)
                OVERWRITE_FIRST.add(self.params[1])
            else:
                if empty and self.params[1] in OVERWRITE_FIRST:  # its slice was not zeroed by a lazy zero_grad
                    G.zero_(tgt)
                    OVERWRITE_FIRST.discard(self.params[1])
                F.gemm_tn_acc(x2, dy2, tgt, colsum_b=tb if fuse_db else None)
            _WGRAD_EPOCH[wid] = GRAD_EPOCH[0]
            dw = ACCUMULATED
        else:
            dw = F.gemm(x2, dy2, ta=True, out_dtype=torch.float32)
        res = [dx, dw]
        if self.has_bias:
            if db_done:
                db = ACCUMULATED
            elif cs_pre is not None and tb is not None:
                G.binary("add", tb, G.reshape(cs_pre, tb.shape), out=tb)
                db = ACCUMULATED
            elif cs_pre is not None:
                db = cs_pre
            elif fuse_db:
                db = ACCUMULATED
            elif tb is not None:
                F.colsum(dy2, out=tb)
                db = ACCUMULATED
            else:
                db = F.colsum(dy2)[0]
            res.append(db)
        return tuple(res)


class Conv2d(Operator):
    """2-D convolution; NCHW logical / NHWC physical; implicit-GEMM kernels."""

    def __init__(self, stride=(1, 1), padding=(0, 0), dilation=(1, 1), group=1, has_bias=False,
                 fuse_relu=False, bn_stats=False, name=None):
        super().__init__(name)
        self.stride, self.padding, self.dilation, self.group = tuple(stride), tuple(padding), tuple(dilation), group
        self.has_bias = has_bias
        self.fuse_relu = fuse_relu
        self.bn_stats = bn_stats  # a training-mode BatchNorm consumes the output: sum its statistics in the epilogue

    def forward(self, x, W, b=None):
        p = self.params[1] if len(self.params) > 1 else None
        w = p.low if (p is not None and p.low is not None and x.dtype == torch.bfloat16) else W
        y = F.conv2d_fwd(x, w, b, self.stride, self.padding, self.dilation, self.group, out_dtype=x.dtype,
                         relu=self.fuse_relu, bn_stats=self.bn_stats and _training())
        xc = getattr(y, "_sg_xconv", None)
        if xc is not None:
            del y._sg_xconv
        if self.requires_grad:
            # an input that needs no gradient (the images) is kept in the
            # converted bf16 NHWC (channel-padded) form the forward built, so
            # the backward does not convert it again
            self.x = xc if (xc is not None and not self.needs_grad(0)) else x
            self.w = w
            self.y = y if self.fuse_relu else None
        return y

    accepts_acc = True
    wants_sole = True  # the identity-sum BN backward needs to be the producer's only consumer

    def backward(self, dy):
        x, w = self.x, self.w
        self.x = self.w = None
        if self.fuse_relu:
            if not getattr(self, "dy_relu_done", False):  # (an LRN consumer may have applied the mask)
                dy = F.relu_bwd_from_y(self.y, dy)
            self.dy_relu_done = False
            self.y = None
        tgt = self.grad_target(1)
        acc = (getattr(self, "acc_into", None) or {}).get(0)
        # input produced by a training BN+ReLU (no residual): its backward
        # reduction is fused into this dgrad's epilogue
        prod = self.src[0][0] if self.src else None
        bnp = None
        wdot = False
        if (isinstance(prod, BatchNorm2d) and prod.relu and getattr(prod, "st", None) is not None
                and getattr(prod, "x", None) is not None):
            if (acc is None and not prod.has_residual and F.BN_WDOT and prod.st.mask is not None
                    and (getattr(self, "sole", None) or {}).get(0, False)
                    and (tgt is None or _WGRAD_EPOCH.get(id(self.params[1])) != GRAD_EPOCH[0])
                    and getattr(prod, "beta", None) is not None and self.group == 1
                    and (F.BN_WDOT_MODE != 2 or tuple(w.shape[2:]) == (1, 1))
                    and self.needs_grad(0) and tuple(self.dilation) == (1, 1)):
                # identity-sum BN backward: this conv's dgrad sums the masked
                # gradient and its wgrad <W, dW>; the BN skips its reduction
                bnp = (prod.x, prod.st, prod.st.mask, prod.gamma, prod.beta)
                wdot = True
            elif acc is None and not prod.has_residual:
                bnp = (prod.x, prod.st)
            elif (acc is not None and prod.has_residual and prod.st.mask is not None
                  and (getattr(self, "acc_last", None) or {}).get(0, False)):
                # residual BN: this dgrad's accumulation completes its output gradient
                bnp = (prod.x, prod.st, prod.st.mask)
        elif (isinstance(prod, (ConvBNAddReLU, ConvBNDualAddReLU)) and getattr(prod, "st", None) is not None
              and prod.st.mask is not None
              and self.group == 1 and tuple(self.dilation) == (1, 1) and self.needs_grad(0)
              and ((acc is not None and (getattr(self, "acc_last", None) or {}).get(0, False))
                   or (acc is None and (getattr(self, "sole", None) or {}).get(0, False)))):
            # the fused residual tail: this dgrad completes its output gradient,
            # so the epilogue writes it masked (g) and sums it per channel
            bnp = ("gmask", prod.st.mask)
        wt_pre, self.wt_pre = getattr(self, "wt_pre", None), None
        tb = self.grad_target(2) if self.has_bias else None
        dx, dw, db = F.conv2d_bwd(x, w, dy, self.stride, self.padding, self.dilation, self.group,
                                  need_dx=self.needs_grad(0), dw_out=tgt, need_db=self.has_bias, dx_acc=acc,
                                  bn_producer=bnp, wt_pre=wt_pre, db_out=tb, bn_wdot=wdot)
        if tgt is not None:
            _WGRAD_EPOCH[id(self.params[1])] = GRAD_EPOCH[0]  # this step's weight gradient is no longer empty
        if acc is not None and getattr(dx, "_sg_absorbed", None) is acc:
            del dx._sg_absorbed
            dx = AccReplace(dx)  # the dgrad summed acc into its own fresh output
        elif acc is not None and (dx is acc or (isinstance(acc, F.LAZY_GRADS) and acc.value is not None
                                                and dx is acc.value)):
            # summed in place into the pending gradient (a lazy residual
            # gradient the dgrad materialised holds the sum as its value)
            dx = ACC_INPLACE
        res = [dx, ACCUMULATED if tgt is not None else dw]
        if self.has_bias:
            res.append(ACCUMULATED if tb is not None else db)  # accumulated into the grad view by the kernel
        return tuple(res)


class BatchNorm2d(Operator):
    """Batch normalisation (+ optional fused ReLU and residual add).
    Inputs: x, gamma, beta[, residual].  Running stats are updated in place.
    dgamma/dbeta are accumulated by the kernel straight into the flat
    gradient buffer when the params live in a ParamStore."""

    def __init__(self, running_mean: torch.Tensor, running_var: torch.Tensor, momentum: float = 0.1,
                 eps: float = 1e-5, relu: bool = False, has_residual: bool = False, name=None,
                 colsum: bool = False):
        super().__init__(name)
        self.rm, self.rv = running_mean, running_var
        self.momentum, self.eps = momentum, eps
        self.relu, self.has_residual = relu, has_residual
        self.colsum = colsum  # the consumer is a fused residual tail: sum the output's columns too

    def forward(self, x, gamma, beta, res=None):
        # ReLU after a residual add: the mask cannot be recomputed from x, so
        # the forward writes it as bits (1/16 of re-reading the bf16 output)
        # (and for the identity-sum backward, F.BN_WDOT: a consuming conv
        # reads these bits instead of x to sum the masked gradient)
        want = self.requires_grad and self.relu and (self.has_residual or (F.BN_WDOT and _training()))
        y, st = F.batchnorm_fwd(x, gamma, beta, self.rm, self.rv, _training(), self.momentum, self.eps, self.relu,
                                res, want_mask=want, want_colsum=self.colsum and self.requires_grad)
        if self.requires_grad:
            self.x, self.gamma, self.st = x, gamma, st
            self.beta = beta if F.BN_WDOT else None
            # the fused output is the ReLU mask only when a residual was added and no bit mask exists
            self.y = y if (want and st.mask is None) else None
        return y

    def backward(self, dy):
        tg, tb = self.grad_target(1), self.grad_target(2)
        dx, dg, db, dres = F.batchnorm_bwd(self.x, dy, self.gamma, self.st, self.y, need_dres=self.has_residual,
                                           relu=self.relu, dg_out=tg, db_out=tb, beta=getattr(self, "beta", None),
                                           lazy_dres=True)
        self.x = self.y = self.st = self.beta = None
        out = [dx, ACCUMULATED if tg is not None else dg, ACCUMULATED if tb is not None else db]
        if self.has_residual:
            out.append(dres)
        return tuple(out)


class ConvBNAddReLU(Operator):
    """out = relu(BN(conv1x1(y, W)) + res): a bottleneck's residual tail as one
    operator (inputs y, W, gamma, beta, res) so its backward can run
    algebraically (F.bnres_bwd, csrc/kernels/bnres.hip): no pass over the conv
    output c or its gradient -- the BN's two sums come from the masked output
    gradient g (written, masked and summed, by the consuming conv's dgrad
    epilogue) and from G = g^T y, the conv's gradients from one two-source
    weight-gradient GEMM ([g | y]^T y) and one two-source data-gradient GEMM
    ([g | y] against [W^T diag(s) | -W^T diag(u) W]).  The residual's gradient
    is g itself.  The forward: on short-K tails the conv runs twice and c is
    never stored (F.bnres_fwd: statistics pass, then BN + residual + ReLU in
    the GEMM epilogue); elsewhere the unfused conv (BN statistics in its
    epilogue) + BN apply; c is not kept either way."""

    wants_sole = True  # the producer BN's identity-sum backward needs this op to be y's only consumer

    def __init__(self, running_mean: torch.Tensor, running_var: torch.Tensor, momentum: float, eps: float,
                 name=None):
        super().__init__(name)
        self.rm, self.rv = running_mean, running_var
        self.momentum, self.eps = momentum, eps

    def forward(self, y, W, gamma, beta, res):
        p = self.params[1] if len(self.params) > 1 else None
        w = p.low if (p is not None and p.low is not None and y.dtype == torch.bfloat16) else W
        r = F.bnres_fwd(y, w, gamma, beta, self.rm, self.rv, _training(), self.momentum, self.eps, res)
        if r is not None:  # c recomputed, never stored
            out, st = r
        else:
            c = F.conv2d_fwd(y, w, None, (1, 1), (0, 0), (1, 1), 1, out_dtype=y.dtype, relu=False,
                             bn_stats=_training())
            out, st = F.batchnorm_fwd(c, gamma, beta, self.rm, self.rv, _training(), self.momentum, self.eps, True,
                                      res, want_mask=self.requires_grad)
        if self.requires_grad:
            self.y, self.w, self.gamma, self.st = y, w, gamma, st
        return out

    def backward(self, dout):
        y, w, gamma, st = self.y, self.w, self.gamma, self.st
        self.y = self.w = self.gamma = self.st = None
        pre = getattr(dout, "_sg_gsum", None)
        if pre is not None and pre[1] is st.mask:
            g, gws = dout, pre[0]  # masked and summed by the consuming conv's dgrad epilogue
            del dout._sg_gsum
        else:
            g, gws = F.bnres_masksum(dout, st.mask)
        # the producer of y: a BN(+ReLU) whose identity-sum backward this op's
        # dgrad epilogue can serve (as Conv2d.backward's wdot path)
        prod = self.src[0][0] if self.src else None
        prod2 = None
        if (isinstance(prod, BatchNorm2d) and prod.relu and not prod.has_residual and F.BN_WDOT
                and getattr(prod, "st", None) is not None and prod.st.mask is not None
                and getattr(prod, "beta", None) is not None and (getattr(self, "sole", None) or {}).get(0, False)
                and self.needs_grad(0)):
            prod2 = (prod.st.mask, prod.gamma, prod.beta)
        tw, tg, tb = self.grad_target(1), self.grad_target(2), self.grad_target(3)
        cs = getattr(getattr(prod, "st", None), "colsum", None) if isinstance(prod, BatchNorm2d) else None
        dy, dw, dg, db = F.bnres_bwd(g, gws, y, w, st, gamma, dw_out=tw, dg_out=tg, db_out=tb, prod2=prod2, cs=cs)
        if tw is not None:
            _WGRAD_EPOCH[id(self.params[1])] = GRAD_EPOCH[0]
        g._sg_fresh = True  # the residual's gradient: the engine may accumulate into it in place
        acc = lambda tgt, v: ACCUMULATED if tgt is not None else v  # noqa: E731
        return dy, acc(tw, dw), acc(tg, dg), acc(tb, db), g


class ConvBNDualAddReLU(Operator):
    """out = relu(BN3(conv1x1(y, W3)) + BNd(conv1x1_s(x, Wd))): a downsample
    bottleneck's tail (main 1x1 conv + BN, strided 1x1 shortcut conv + BN) as
    one operator, inputs y, W3, gamma3, beta3, x, Wd, gammad, betad.  Both
    branches' backward runs algebraically as ConvBNAddReLU's (F.bnres_bwd,
    twice, on the same masked output gradient g): no pass over either conv
    output or its gradient -- the fused two-BN backward (bn_bwd2: a reduction
    and an apply pass over g, c3 and cd, writing dc3 and dcd) disappears.  A
    strided shortcut reads x at every s-th pixel: those pixels are gathered
    once in the forward (F.strided_pick), so the shortcut is a plain GEMM and
    its input gradient is placed back on the full grid (F.strided_place).
    Reference block: src/worker/layer.cc:75-122 (conv + BN per layer)."""

    wants_sole = True  # (y's producer BN: the identity-sum backward, as ConvBNAddReLU)

    def __init__(self, bn3, bnd, stride: int, name=None):
        super().__init__(name)
        self.p3 = (bn3.running_mean.data, bn3.running_var.data, 1.0 - bn3.momentum, bn3.eps)
        self.pd = (bnd.running_mean.data, bnd.running_var.data, 1.0 - bnd.momentum, bnd.eps)
        self.stride = stride

    def _low(self, i, W, like):
        p = self.params[i] if len(self.params) > i else None
        return p.low if (p is not None and p.low is not None and like.dtype == torch.bfloat16) else W

    def forward(self, y, W3, g3, b3, x, Wd, gd, bd):
        w3, wd = self._low(1, W3, y), self._low(5, Wd, x)
        xs = x if self.stride == 1 else F.strided_pick(x, self.stride)
        tr = _training()
        rm, rv, mom, eps = self.p3
        rm2, rv2, mom2, eps2 = self.pd
        r = (F.bnres_dual_fwd(y, w3, g3, b3, rm, rv, mom, eps, xs, wd, gd, bd, rm2, rv2, mom2, eps2, tr)
             if self.stride == 1 else None)
        if r is not None:  # both conv outputs recomputed, never stored
            out, st3, std = r
        else:
            c3 = F.conv2d_fwd(y, w3, None, (1, 1), (0, 0), (1, 1), 1, out_dtype=y.dtype, bn_stats=tr)
            cd = F.conv2d_fwd(xs, wd, None, (1, 1), (0, 0), (1, 1), 1, out_dtype=y.dtype, bn_stats=tr)
            out, st3, std = F.dual_bn_add_relu_fwd(c3, g3, b3, rm, rv, cd, gd, bd, rm2, rv2, tr, mom, eps, mom2,
                                                   eps2)
        if self.requires_grad:
            self.st = st3  # (the ReLU mask: the consuming conv's dgrad epilogue writes g with it)
            self.saved = (y, w3, g3, xs, tuple(x.shape), wd, gd, std)
        return out

    def backward(self, dout):
        y, w3, g3, xs, xshape, wd, gd, std = self.saved
        st3 = self.st
        self.saved = self.st = None
        pre = getattr(dout, "_sg_gsum", None)
        if pre is not None and pre[1] is st3.mask:
            g, gws = dout, pre[0]  # masked and summed by the consuming conv's dgrad epilogue
            del dout._sg_gsum
        else:
            g, gws = F.bnres_masksum(dout, st3.mask)
        prod = self.src[0][0] if self.src else None
        prod2 = None
        if (isinstance(prod, BatchNorm2d) and prod.relu and not prod.has_residual and F.BN_WDOT
                and getattr(prod, "st", None) is not None and prod.st.mask is not None
                and getattr(prod, "beta", None) is not None and (getattr(self, "sole", None) or {}).get(0, False)
                and self.needs_grad(0)):
            prod2 = (prod.st.mask, prod.gamma, prod.beta)
        cs = getattr(getattr(prod, "st", None), "colsum", None) if isinstance(prod, BatchNorm2d) else None
        t = [self.grad_target(i) for i in (1, 2, 3, 5, 6, 7)]
        dy, dw3, dg3, db3 = F.bnres_bwd(g, gws, y, w3, st3, g3, dw_out=t[0], dg_out=t[1], db_out=t[2], prod2=prod2,
                                        cs=cs)
        dxs, dwd, dgd, dbd = F.bnres_bwd(g, gws, xs, wd, std, gd, dw_out=t[3], dg_out=t[4], db_out=t[5])
        for i, tg in ((1, t[0]), (5, t[3])):
            if tg is not None:
                _WGRAD_EPOCH[id(self.params[i])] = GRAD_EPOCH[0]
        dx = None
        if self.needs_grad(4):
            # (strided: kept compact -- the block's conv1 dgrad epilogue adds it)
            dx = dxs if self.stride == 1 else (F.StridedGrad(dxs, self.stride, xshape) if F.STRIDED_LAZY
                                               else F.strided_place(dxs, xshape, self.stride))
        acc = lambda tgt, v: ACCUMULATED if tgt is not None else v  # noqa: E731
        return (dy, acc(t[0], dw3), acc(t[1], dg3), acc(t[2], db3), dx, acc(t[3], dwd), acc(t[4], dgd),
                acc(t[5], dbd))


class DualBNAddReLU(Operator):
    """y = relu(BN(x) + BN2(x2)): a residual block's output BN with a
    downsample shortcut (conv + BN), fused -- the shortcut BN's output and
    the residual gradient are never materialised.  Inputs x, gamma, beta, x2,
    gamma2, beta2."""

    def __init__(self, bn1, bn2, name=None):
        super().__init__(name)
        self.p1 = (bn1.running_mean.data, bn1.running_var.data, 1.0 - bn1.momentum, bn1.eps)
        self.p2 = (bn2.running_mean.data, bn2.running_var.data, 1.0 - bn2.momentum, bn2.eps)

    def forward(self, x, gamma, beta, x2, gamma2, beta2):
        rm, rv, mom, eps = self.p1
        rm2, rv2, mom2, eps2 = self.p2
        y, st, st2 = F.dual_bn_add_relu_fwd(x, gamma, beta, rm, rv, x2, gamma2, beta2, rm2, rv2, _training(), mom, eps,
                                            mom2, eps2)
        if self.requires_grad:
            self.saved = (x, gamma, st, x2, gamma2, st2)
        return y

    def backward(self, dy):
        x, gamma, st, x2, gamma2, st2 = self.saved
        self.saved = None
        t = [self.grad_target(i) for i in (1, 2, 4, 5)]
        dx, dg, db, dx2, dg2, db2 = F.dual_bn_add_relu_bwd(x, dy, gamma, st, x2, gamma2, st2, *t)
        acc = lambda tgt, v: ACCUMULATED if tgt is not None else v  # noqa: E731
        return dx, acc(t[0], dg), acc(t[1], db), dx2, acc(t[2], dg2), acc(t[3], db2)


class BnReluMaxPool(Operator):
    """max_pool(relu(BatchNorm(x))) as one forward pass (a ResNet stem): the
    full-resolution BN output is never written.  Inputs x, gamma, beta; the
    backward gathers the pooled gradient through the argmax, then runs the BN
    backward with the ReLU mask recomputed from x."""

    def __init__(self, running_mean: torch.Tensor, running_var: torch.Tensor, momentum: float, eps: float,
                 kernel, stride, padding, name=None):
        super().__init__(name)
        self.rm, self.rv = running_mean, running_var
        self.momentum, self.eps = momentum, eps
        self.kernel, self.stride, self.padding = tuple(kernel), tuple(stride), tuple(padding)

    def forward(self, x, gamma, beta):
        y, arg, st = F.bn_relu_maxpool_fwd(x, gamma, beta, self.rm, self.rv, _training(), self.momentum, self.eps,
                                           self.kernel, self.stride, self.padding)
        if self.requires_grad:
            self.x, self.gamma, self.st, self.arg = x, gamma, st, arg
        return y

    def backward(self, dy):
        tg, tb = self.grad_target(1), self.grad_target(2)
        dx, dg, db = F.bn_relu_maxpool_bwd(self.x, dy, self.arg, self.gamma, self.st, self.kernel, self.stride,
                                           self.padding, dg_out=tg, db_out=tb)
        self.x = self.st = self.arg = None
        return dx, ACCUMULATED if tg is not None else dg, ACCUMULATED if tb is not None else db


class Pooling2d(Operator):
    def __init__(self, kernel, stride, padding=(0, 0), is_max=True, count_include_pad=True, ceil_mode=False,
                 name=None):
        super().__init__(name)
        self.kernel, self.stride, self.padding = tuple(kernel), tuple(stride), tuple(padding)
        self.is_max, self.cip, self.ceil = is_max, count_include_pad, ceil_mode

    def forward(self, x):
        y, arg = F.pool2d_fwd(x, self.kernel, self.stride, self.padding, self.is_max, self.cip, self.ceil)
        if self.requires_grad:
            self.xs, self.xl, self.arg = x.shape, x, arg
        return y

    def backward(self, dy):
        dx = F.pool2d_bwd(self.xs, self.xl, dy, self.arg, self.kernel, self.stride, self.padding, self.is_max,
                          self.cip, self.ceil)
        self.xl = self.arg = None
        return dx


class GlobalAveragePool(Operator):
    """[N,C,H,W] -> [N,C] (SINGA's GlobalAveragePool keeps [N,C,1,1]; set keepdims)."""

    def __init__(self, keepdims: bool = False, name=None):
        super().__init__(name)
        self.keepdims = keepdims

    def forward(self, x):
        if self.requires_grad:
            self.xs = x.shape
        y = F.global_avgpool_fwd(x)
        return y.reshape(y.shape[0], y.shape[1], 1, 1) if self.keepdims else y

    def backward(self, dy):
        return F.global_avgpool_bwd(G.contiguous(G.reshape(dy, (dy.shape[0], dy.shape[1]))), self.xs)


class LRN(Operator):
    """Across-channel local response normalisation (reference kLRN,
    src/worker/layer.cc:331-378)."""

    def __init__(self, size=5, alpha=1e-4, beta=0.75, k=1.0, name=None):
        super().__init__(name)
        self.size, self.alpha, self.beta, self.k = size, alpha, beta, k

    wants_sole = True

    def forward(self, x):
        y, norm = F.lrn_fwd(x, self.size, self.alpha, self.beta, self.k)
        if self.requires_grad:
            self.x, self.norm = x, norm
        return y

    def backward(self, dy):
        # input from a conv with fused ReLU whose only consumer is this LRN:
        # apply the ReLU mask (x > 0, x being that ReLU's output) in the LRN
        # backward kernel and tell the conv to skip its relu_bwd pass
        prod = self.src[0][0] if self.src else None
        fold = (isinstance(prod, Conv2d) and prod.fuse_relu and getattr(prod, "y", None) is not None
                and prod.y is self.x and (getattr(self, "sole", None) or {}).get(0, False))
        dx = F.lrn_bwd(self.x, dy, self.norm, self.size, self.alpha, self.beta, self.k, relu_mask=fold)
        if fold and getattr(dx, "_sg_relu_done", False):
            prod.dy_relu_done = True
        self.x = self.norm = None
        return dx


class Dropout(Operator):
    """Inverted dropout; identity when not training (fixes reference quirk
    #9: the kDropout layer masked at test time, src/worker/layer.cc:142-152)."""

    def __init__(self, ratio: float = 0.5, seed_source=None, name=None):
        super().__init__(name)
        self.ratio = ratio
        self.seed_source = seed_source

    def forward(self, x):
        if not _training() or self.ratio <= 0.0:
            self.mask = None
            return x
        dev = self.seed_source
        seed, off = dev.next_rng(x.numel()) if dev is not None else (0, 0)
        ep = dev.rng_epoch() if dev is not None and x.is_cuda else None
        y, self.mask = F.dropout_fwd(x, self.ratio, seed, off, ep)
        return y

    def backward(self, dy):
        if self.mask is None:
            return dy
        dx = F.dropout_bwd(dy, self.mask, self.ratio)
        self.mask = None
        return dx


class SoftMax(Operator):
    def __init__(self, axis: int = 1, name=None):
        super().__init__(name)
        self.axis = axis

    def forward(self, x):
        y = F.softmax(x, self.axis)
        if self.requires_grad:
            self.y = y
        return y

    def backward(self, dy):
        dx = F.softmax_bwd(self.y, dy, self.axis)
        self.y = None
        return dx


class SoftMaxCrossEntropy(Operator):
    """Fused softmax + cross-entropy; loss = mean over the batch.  Target is
    either class ids or a one-hot / probability matrix.  Also records top-k
    accuracy in ``self.correct`` (the reference's loss-layer metric)."""

    def __init__(self, t: Optional[torch.Tensor] = None, topk: int = 1, name=None):
        super().__init__(name)
        self.t = t
        self.topk = topk

    def forward(self, x, t=None):
        t = self.t if t is None else t
        loss, correct, dx = F.softmax_xent(x, t, self.topk, need_grad=self.requires_grad)
        self.dx = dx
        self.correct = correct
        self.per_row = loss
        self.nt = 2 if self.t is None and t is not None else 1
        return G.reduce(loss, None, "mean", out_dtype=torch.float32)

    def backward(self, dy=None):
        dx = self.dx
        self.dx = None
        if not is_unit(dy):
            dx = G.binary("mul", dx, dy, out_dtype=dx.dtype)
        return (dx, None) if len(self.src) == 2 else dx


class CrossEntropy(Operator):
    """Cross entropy over probabilities: -sum(t * log(p)) / B."""

    def forward(self, p, t):
        B = p.shape[0]
        if t.dim() == 1 or not t.is_floating_point():  # class ids -> one-hot rows
            ids = G.reshape(G.to(t, torch.int64), (-1, 1))
            tt = G.scatter_elements(G.zeros(p.shape, torch.float32, p.device), 1, ids,
                                    G.full(ids.shape, 1.0, torch.float32, p.device))
        else:
            tt = G.to(t, torch.float32)
        lp = F.unary("log", G.clamp_affine(G.to(p, torch.float32), lo=1e-30))
        if self.requires_grad:
            self.p, self.tt = p, tt
        return F.unary("scale", G.reduce(G.binary("mul", tt, lp), None, "sum", out_dtype=torch.float32), -1.0 / B)

    def backward(self, dy=None):
        B = self.p.shape[0]
        # d/dp = -t / clamp(p) / B
        g = G.binary("div", self.tt, G.clamp_affine(G.to(self.p, torch.float32), lo=1e-30), alpha=-1.0 / B)
        if dy is not None and not is_unit(dy):
            g = G.binary("mul", g, dy)
        return G.to(g, self.p.dtype), None


class MeanSquareError(Operator):
    """sum((x - t)^2) / (2B)."""

    def forward(self, x, t):
        d = G.binary("sub", x, t, out_dtype=torch.float32)
        if self.requires_grad:
            self.d = d
        return F.unary("scale", G.reduce(d, None, "sumsq", out_dtype=torch.float32), 1.0 / (2.0 * x.shape[0]))

    def backward(self, dy=None):
        g = F.unary("scale", self.d, 1.0 / self.d.shape[0])
        if dy is not None and not is_unit(dy):
            g = G.binary("mul", g, dy)
        return g, None


class BinaryCrossEntropy(Operator):
    """-mean(t log p + (1 - t) log(1 - p)), p clamped to [1e-7, 1 - 1e-7]."""

    def forward(self, x, t):
        p = G.clamp_affine(G.to(x, torch.float32), lo=1e-7, hi=1 - 1e-7)
        tf = G.to(t, torch.float32)
        if self.requires_grad:
            self.p, self.t = p, tf
        lp = F.unary("log", p)
        l1p = F.unary("log", G.clamp_affine(p, -1.0, 1.0))  # log(1 - p)
        s = G.binary("add", G.binary("mul", tf, lp), G.binary("mul", F.unary("adds", F.unary("neg", tf), 1.0), l1p))
        return F.unary("neg", G.reduce(s, None, "mean", out_dtype=torch.float32))

    def backward(self, dy=None):
        p, t = self.p, self.t
        # (p - t) / (p (1 - p)) / n
        den = G.binary("mul", p, G.clamp_affine(p, -1.0, 1.0))
        g = G.binary("div", G.binary("sub", p, t), den, alpha=1.0 / p.numel())
        if dy is not None and not is_unit(dy):
            g = G.binary("mul", g, dy)
        return g, None


class DropAddLayerNorm(Operator):
    """y = LayerNorm(x + dropout(a)): a transformer block's residual tail as
    one operator (inputs x, a, gamma, beta).  Forward: one pass writing the
    sum s (the backward's input), the dropout byte mask and y -- instead of
    dropout, add and LayerNorm passes; the mask comes from the dropout
    kernel's Philox stream for the same (seed, offset) draw, so the numbers
    are the unfused chain's.  Backward: one pass writing ds (x's gradient)
    and da (a's, through the mask) and summing da's columns, handed to the
    producing Linear as its bias gradient (``da._sg_colsum``: no separate
    column-sum pass over da)."""

    wants_sole = True  # (the producing Linear's bias gradient is summed here when this op is a's only consumer)

    def __init__(self, ratio: float, seed_source, eps: float, name=None):
        super().__init__(name)
        self.ratio, self.seed_source, self.eps = ratio, seed_source, eps

    def forward(self, x, a, g, b):
        ratio, seed, off, ep = 0.0, 0, 0, None
        if _training() and self.ratio > 0.0:
            dev = self.seed_source
            seed, off = dev.next_rng(a.numel()) if dev is not None else (0, 0)
            ep = dev.rng_epoch() if dev is not None and a.is_cuda else None
            ratio = self.ratio
        y, s, mask, mean, rstd = F.drop_add_layernorm_fwd(x, a, g, b, self.eps, ratio, seed, off, ep)
        if self.requires_grad:
            self.saved = (s, g, mean, rstd, mask, ratio)
        return y

    def _producer_bias(self):
        return producer_bias(self, 1)

    def backward(self, dy):
        s, g, mean, rstd, mask, ratio = self.saved
        self.saved = None
        tg, tb = self.grad_target(2), self.grad_target(3)
        prod, cs_to = self._producer_bias()
        if cs_to is not None and cs_to.numel() != s.shape[-1]:
            prod = cs_to = None
        ds, da, dg, db, cs = F.drop_add_layernorm_bwd(s, dy, g, mean, rstd, mask, ratio, dg_acc=tg, db_acc=tb,
                                                      cs_acc=cs_to)
        ds._sg_fresh = True  # (a buffer of its own: x's other consumer may add into it in place)
        if prod is not None:
            prod.db_done = True  # da's column sums went straight into the producer's bias gradient
        else:
            da._sg_colsum = cs
        acc = lambda tgt, v: ACCUMULATED if tgt is not None else v  # noqa: E731
        return ds, da, acc(tg, dg), acc(tb, db)


class LayerNorm(Operator):
    def __init__(self, eps: float = 1e-5, name=None):
        super().__init__(name)
        self.eps = eps

    def forward(self, x, g=None, b=None):
        y, mean, rstd = F.layernorm_fwd(x, g, b, self.eps)
        if self.requires_grad:
            self.x, self.g, self.mean, self.rstd = x, g, mean, rstd
        return y

    def backward(self, dy):
        tg = self.grad_target(1) if len(self.src) > 1 else None
        tb = self.grad_target(2) if len(self.src) > 2 else None
        # the kernel accumulates dgamma / dbeta straight into the flat-store views
        dx, dg, db = F.layernorm_bwd(self.x, dy.contiguous(), self.g, self.mean, self.rstd, dg_acc=tg, db_acc=tb)
        self.x = None
        out = [dx]
        if len(self.src) > 1:
            for i, gg, t in ((1, dg, tg), (2, db, tb)):
                if i >= len(self.src):
                    break
                if t is not None and gg is not None:
                    if gg is not t:
                        G.binary("add", t, G.reshape(gg, t.shape), out=t)
                    out.append(ACCUMULATED)
                else:
                    out.append(gg)
        return tuple(out) if len(out) > 1 else out[0]


class Cast(Operator):
    def __init__(self, to, name=None):
        super().__init__(name)
        self.to = to

    def forward(self, x):
        self.from_dtype = x.dtype
        return F.cast(x, self.to) if x.is_floating_point() else x.to(self.to)

    def backward(self, dy):
        if not self.from_dtype.is_floating_point:
            return None
        dx = F.cast(dy, self.from_dtype)
        cs = getattr(dy, "_sg_colsum", None)  # (column sums a producer already took: still dx's)
        if cs is not None and dx is not dy:
            dx._sg_colsum = cs
        return dx


class ToChannelsLast(Operator):
    """Layout change NCHW -> NHWC memory (no logical change); GPU entry op."""

    def __init__(self, dtype=None, name=None):
        super().__init__(name)
        self.dtype = dtype

    def forward(self, x):
        self.from_dtype = x.dtype
        if x.dim() != 4:
            return x.to(self.dtype) if self.dtype else x
        return x.to(dtype=self.dtype or x.dtype, memory_format=torch.channels_last)

    def backward(self, dy):
        return dy.to(self.from_dtype)


class Reshape(Operator):
    def __init__(self, shape, name=None):
        super().__init__(name)
        self.shape = list(shape)

    def forward(self, x):
        self.in_shape = x.shape
        shape = [x.shape[i] if s == 0 and i < x.dim() else s for i, s in enumerate(self.shape)]
        return G.reshape(x, shape)

    def backward(self, dy):
        return G.reshape(dy, self.in_shape)


class Flatten(Operator):
    def __init__(self, axis: int = 1, name=None):
        super().__init__(name)
        self.axis = axis

    def forward(self, x):
        self.in_shape = x.shape
        a = self.axis % _b.max(x.dim(), 1) if x.dim() else 0
        lead = int(np.prod(x.shape[:a])) if a > 0 else 1
        return G.reshape(x, (lead, -1))

    def backward(self, dy):
        return G.reshape(dy, self.in_shape)


class Attention(Operator):
    """Scaled dot-product attention softmax(q k^T * scale + mask) v over
    [..., S, D] heads (mask: additive, non-differentiable).  bf16 on the GPU
    runs batched MFMA GEMMs + the softmax kernels (functional.attention_*)."""

    def __init__(self, scale: Optional[float] = None, name=None):
        super().__init__(name)
        self.scale = scale

    def forward(self, q, k, v, mask=None):
        o, p = F.attention_fwd(q, k, v, mask, self.scale)
        if self.requires_grad:
            self.saved = (q, k, v, p)
        return o

    def backward(self, do):
        q, k, v, p = self.saved
        self.saved = None
        dq, dk, dv = F.attention_bwd(q, k, v, p, do.contiguous(), self.scale)
        return (dq, dk, dv) + ((None,) if len(self.src) == 4 else ())


BIAS_INPLACE = os.environ.get("SINGA_AMD_BIAS_INPLACE", "1") != "0"  # (A/B switch)
# a Linear's data-gradient GEMM applies the derivative of a standalone
# activation op that feeds it (GELU between BERT's fc1 and fc2)
ACT_GRAD_FUSE = os.environ.get("SINGA_AMD_ACT_GRAD_FUSE", "1") != "0"  # (A/B switch)


def producer_bias(op: Operator, i: int):
    """(Linear, its fp32 bias-gradient view) when input i of ``op`` is the
    output of a plain Linear (bias, no fused activation) whose gradient comes
    from ``op`` alone: ``op``'s backward may then sum that gradient's columns
    straight into the bias gradient (and set ``Linear.db_done``), else
    (None, None)."""
    src = op.src[i][0] if len(op.src) > i and BIAS_INPLACE else None
    if not (isinstance(src, Linear) and src.has_bias and src.act is None
            and (getattr(op, "sole", None) or {}).get(i, False)):
        return None, None
    tb = src.grad_target(2)
    ok = tb is not None and tb.is_cuda and tb.dtype == torch.float32 and tb.is_contiguous()
    return (src, tb) if ok else (None, None)


class QKVAttention(Operator):
    """Multi-head attention fed by the fused q/k/v projection: qkv [B, S,
    3*H*D] -> [B, S, H*D].  Equivalent to split-heads -> Attention ->
    merge-heads, but the batched MFMA GEMMs address each head in place
    (functional.attention_qkv_*), so neither direction copies the heads."""

    wants_sole = True  # (the fused backward sums the q/k/v projection's bias gradient when qkv has no other consumer)

    def __init__(self, heads: int, scale: Optional[float] = None, name=None):
        super().__init__(name)
        self.heads, self.scale = heads, scale

    def forward(self, qkv, mask=None):
        o, p = F.attention_qkv_fwd(qkv, self.heads, mask, self.scale)
        if self.requires_grad:
            self.saved = (qkv, p)
        return o

    def backward(self, do):
        qkv, p = self.saved
        self.saved = None
        prod, db = self._producer_bias()
        if not F.fattn_bias_ok(p, db, qkv.shape[-1]):
            prod = db = None
        dqkv = F.attention_qkv_bwd(qkv, p, do, self.heads, self.scale, db_acc=db)
        if prod is not None:
            prod.db_done = True  # d(qkv)'s column sums went straight into the projection's bias gradient
        return (dqkv, None) if len(self.src) == 2 else dqkv

    def _producer_bias(self):
        return producer_bias(self, 0)


def attention(q, k, v, mask=None, scale=None):
    return Attention(scale)(q, k, v, mask) if mask is not None else Attention(scale)(q, k, v)


# ===========================================================================
# functional API (singa.autograd.xxx)
# ===========================================================================
def relu(x):
    return ReLU()(x)


def sigmoid(x):
    return Sigmoid()(x)


def tanh(x):
    return Tanh()(x)


def stanh(x):
    return STanh()(x)


def gelu(x):
    return Gelu()(x)


def softplus(x):
    return SoftPlus()(x)


def exp(x):
    return Exp()(x)


def log(x):
    return Log()(x)


def abs(x):  # noqa: A001
    return Abs()(x)


def sqrt(x):
    return Sqrt()(x)


def reciprocal(x):
    return Reciprocal()(x)


def negative(x):
    return Negative()(x)


def sign(x):
    return Sign()(x)


def square(x):
    return Square()(x)


def leakyrelu(x, a=0.01):
    return LeakyRelu(a)(x)


def elu(x, alpha=1.0):
    return Elu(alpha)(x)


def selu(x, alpha=1.67326, gamma=1.0507):
    return SeLU(alpha, gamma)(x)


def identity(x):
    return Identity()(x)


def _t(x, like: Tensor):
    if isinstance(x, Tensor):
        return x
    return Tensor(device=like.device, data=torch.as_tensor(x, dtype=like.dtype, device=like.data.device),
                  requires_grad=False)


def add(a, b):
    return Add()(a, _t(b, a))


def add_relu(a, b):
    return Add(relu=True)(a, b)


def sub(a, b):
    return Sub()(a, _t(b, a))


def mul(a, b):
    return Mul()(a, _t(b, a))


def div(a, b):
    return Div()(a, _t(b, a))


def pow(a, b):  # noqa: A001
    return Pow()(a, _t(b, a))


def matmul(a, b):
    return Matmul()(a, b)


def add_bias(x, b, axis=0):
    return AddBias(axis)(x, b)


def linear(x, W, b=None, act=None):
    return Linear(True, act=act)(x, W, b) if b is not None else Linear(False, act=act)(x, W)


def softmax(x, axis=1):
    return SoftMax(axis)(x)


def softmax_cross_entropy(x, t, topk=1):
    return SoftMaxCrossEntropy(topk=topk)(x, t)


def cross_entropy(y, t):
    return CrossEntropy()(y, t)


def mse_loss(x, t):
    return MeanSquareError()(x, t)


def binary_cross_entropy(x, t):
    return BinaryCrossEntropy()(x, t)


def reshape(x, shape):
    return Reshape(shape)(x)


def flatten(x, axis=1):
    return Flatten(axis)(x)


def dropout(x, ratio=0.5):
    return Dropout(ratio, x.device)(x)


def cast(x, to):
    return Cast(to)(x)


def layer_norm(x, g=None, b=None, eps=1e-5):
    args = [a for a in (g, b) if a is not None]
    return LayerNorm(eps)(x, *args)


class Fn(Operator):
    """A glue operator whose forward and backward are plain functions over
    raw tensors built from native kernels (:mod:`singa_amd.ops.glue` /
    :mod:`singa_amd.ops.functional`): ``fwd(*xs) -> (ys, ctx)`` and
    ``bwd(ctx, *dys) -> dxs`` (one entry per input, None if none).  On the
    GPU every data movement is a hand-written kernel; PyTorch runs only on
    CPU tensors (the CppCPU reference).  ``onnx`` is the sonnx export spec."""

    def __init__(self, fwd: Callable, bwd: Optional[Callable] = None, onnx: Optional[dict] = None, name=None):
        super().__init__(name)
        self.fwd, self.bwd, self.onnx = fwd, bwd, onnx

    def forward(self, *xs):
        ys, ctx = self.fwd(*xs)
        self.ctx = ctx if self.requires_grad else None
        return ys

    def backward(self, *dys):
        if self.bwd is None:
            return tuple(None for _ in self.src)
        r = _as_tuple(self.bwd(self.ctx, *dys))
        self.ctx = None
        return r


def _ox(op, attrs=None, inputs=None, n_in=1):
    """sonnx export spec; default inputs: the op's tensor inputs in order."""
    return {"op": op, "attrs": attrs or {}, "inputs": inputs if inputs is not None else
            [("in", i) for i in range(n_in)]}


def transpose(x, shape=None):
    perm = tuple(shape) if shape is not None else tuple(reversed(range(x.ndim())))
    inv = tuple(int(i) for i in np.argsort(perm))
    return Fn(lambda a: (a.permute(*perm), None), lambda c, d: d.permute(*inv),
              onnx=_ox("Transpose", {"perm": list(perm)}))(x)


def _reshape_fn(x, shape, onnx):
    ins = tuple(x.shape)
    return Fn(lambda a: (G.reshape(a, shape), None), lambda c, d: G.reshape(d, ins), onnx=onnx)(x)


def squeeze(x, axis=None):
    ax = None if axis is None else ([axis] if isinstance(axis, int) else list(axis))
    spec = _ox("Squeeze") if ax is None else _ox("Squeeze", inputs=[("in", 0), ("const", np.asarray(ax, np.int64))])
    nd = len(x.shape)
    axs = [a % nd for a in ax] if ax is not None else [k for k, s in enumerate(x.shape) if s == 1]
    shape = [s for k, s in enumerate(x.shape) if not (k in axs and s == 1)]
    return _reshape_fn(x, shape, spec)


def unsqueeze(x, axis):
    ax = [axis] if isinstance(axis, int) else list(axis)
    shape = list(x.shape)
    for d in sorted(a % (len(shape) + len(ax)) for a in ax):
        shape.insert(d, 1)
    return _reshape_fn(x, shape, _ox("Unsqueeze", inputs=[("in", 0), ("const", np.asarray(ax, np.int64))]))


def cat(xs, axis=0):
    sizes = [x.shape[axis] for x in xs]

    def bwd(c, d):
        out, o = [], 0
        for n in sizes:
            out.append(d.narrow(axis, o, n))
            o += n
        return tuple(out)
    return Fn(lambda *a: (G.cat(a, axis), None), bwd, onnx=_ox("Concat", {"axis": axis}, n_in=len(xs)))(*xs)


concat = cat


def split(x, axis, parts):
    parts = list(parts)
    return Fn(lambda a: (tuple(torch.split(a, parts, dim=axis)), a),
              lambda a, *ds: G.scatter_slices(ds, parts, axis, a),
              onnx=_ox("Split", {"axis": axis}, [("in", 0), ("const", np.asarray(parts, np.int64))]))(x)


def slice(x, starts, ends, axes=None, steps=None):  # noqa: A001
    axes = axes if axes is not None else list(range(len(starts)))
    steps = steps if steps is not None else [1] * len(starts)

    def index(a):
        idx = [builtins_slice(None)] * a.dim()
        for s, e, ax, st in zip(starts, ends, axes, steps):
            if st <= 0:
                raise NotImplementedError("slice: only positive steps")
            n = a.shape[ax]
            e = _b.min(e, n) if e >= 0 else e
            idx[ax] = builtins_slice(s, e, st)
        return tuple(idx)

    def fwd(a):
        return a[index(a)], (a.shape, a.dtype, a.device)

    def bwd(c, d):
        shp, dt, dev = c
        g = G.zeros(shp, d.dtype, dev)
        G.copy_(g[index(g)], d)
        return g
    big = 2 ** 62
    spec = _ox("Slice", inputs=[("in", 0), ("const", np.asarray(starts, np.int64)),
                                ("const", np.asarray([e if e < big else big for e in ends], np.int64)),
                                ("const", np.asarray(axes, np.int64)), ("const", np.asarray(steps, np.int64))])
    return Fn(fwd, bwd, onnx=spec)(x)


builtins_slice = _b.slice


def gather(x, axis, indices):
    host = np.asarray(indices) if not isinstance(indices, torch.Tensor) else None
    idx = torch.as_tensor(indices, device=x.data.device).long()
    spec = None
    if _TRACE:  # sonnx export only (the host copy of a device index would sync)
        spec = _ox("Gather", {"axis": axis}, [("in", 0), ("const", host if host is not None else idx.cpu().numpy())])

    def bwd(c, d):
        shp, dt = c
        ax = axis % len(shp)
        g = G.zeros(shp, torch.float32, d.device)
        G.index_add_(g, ax, idx.reshape(-1), G.reshape(d, shp[:ax] + (idx.numel(),) + shp[ax + 1:]))
        return g if dt == torch.float32 else G.to(g, dt)
    return Fn(lambda a: (G.index_select(a, axis, idx), (tuple(a.shape), a.dtype)), bwd, onnx=spec)(x)


def tile(x, repeats):
    reps = list(repeats)
    return Fn(lambda a: (G.tile(a, reps), tuple(a.shape)), lambda shp, d: G.tile_backward(d, reps, shp),
              onnx=_ox("Tile", inputs=[("in", 0), ("const", np.asarray(repeats, np.int64))]))(x)


def expand(x, shape):
    shape = tuple(shape)
    return Fn(lambda a: (a.expand(*shape), tuple(a.shape)), lambda shp, d: G.sum_to(d, shp),
              onnx=_ox("Expand", inputs=[("in", 0), ("const", np.asarray(shape, np.int64))]))(x)


def pad(x, mode="constant", pads=None, constant=0.0):
    n = x.ndim()
    half = len(pads) // 2
    before, after = list(pads[:half]), list(pads[half:])
    before += [0] * (n - len(before))
    after += [0] * (n - len(after))
    spec = _ox("Pad", {"mode": mode}, [("in", 0), ("const", np.asarray(pads, np.int64)),
                                        ("const", np.asarray(constant, np.float32))])
    return Fn(lambda a: (G.pad(a, before, after, mode, float(constant)), tuple(a.shape)),
              lambda shp, d: G.pad_backward(d, shp, before, mode), onnx=spec)(x)


def clip(x, min=None, max=None):  # noqa: A002
    lo = -math.inf if min is None else float(min)
    hi = math.inf if max is None else float(max)
    ins = [("in", 0), ("const", np.asarray(-3.4e38 if min is None else min, np.float32)),
           ("const", np.asarray(3.4e38 if max is None else max, np.float32))]
    # gradient passes where lo <= x <= hi (closed interval, as torch.clamp)
    return Fn(lambda a: (G.clamp_affine(a, 1.0, 0.0, lo, hi), a),
              lambda a, d: G.where(G.binary("and", G.binary("ge", a, lo), G.binary("le", a, hi)), d,
                                   G.zeros((), d.dtype, d.device)),
              onnx=_ox("Clip", inputs=ins))(x)


def where(x, y, condition):
    c = condition.data if isinstance(condition, Tensor) else torch.as_tensor(condition)
    spec = _ox("Where", inputs=[("const", c.bool().cpu().numpy()), ("in", 0), ("in", 1)]) if _TRACE else None

    def fwd(a, b):
        cc = c.to(a.device) if c.device != a.device else c
        return G.where(cc, a, b), (cc, tuple(a.shape), tuple(b.shape))

    def bwd(ctx, d):
        cc, sa, sb = ctx
        z = G.zeros((), d.dtype, d.device)
        return G.sum_to(G.where(cc, d, z), sa), G.sum_to(G.where(cc, z, d), sb)
    return Fn(fwd, bwd, onnx=spec)(x, y)


def _reduce_op(x, axes, keepdims, op, spec):
    def fwd(a):
        return G.reduce(a, axes, op, bool(keepdims), out_dtype=a.dtype if a.is_floating_point() else None), \
            (tuple(a.shape), a.dtype)

    def bwd(ctx, d):
        shp, dt = ctx
        nd = len(shp)
        ax = list(range(nd)) if axes is None else [a % nd for a in axes]
        kshape = [1 if k in ax else s for k, s in enumerate(shp)]
        g = G.expand(G.reshape(d, kshape), shp)
        if op == "mean":
            g = F.unary("scale", g, 1.0 / _b.max(1, int(np.prod([shp[k] for k in ax]))))
        return G.to(g, dt) if g.dtype != dt else g
    return Fn(fwd, bwd, onnx=spec)(x)


def reduce_sum(x, axes=None, keepdims=1):
    ins = [("in", 0)] + ([("const", np.asarray(axes, np.int64))] if axes is not None else [])
    return _reduce_op(x, axes, keepdims if axes is not None else 0, "sum",
                      _ox("ReduceSum", {"keepdims": int(keepdims) if axes is not None else 0}, ins))


def reduce_mean(x, axes=None, keepdims=1):
    at = {"keepdims": int(keepdims) if axes is not None else 0}
    if axes is not None:
        at["axes"] = list(axes)
    return _reduce_op(x, axes, keepdims if axes is not None else 0, "mean", _ox("ReduceMean", at))


def _nary(xs, op, spec):
    """sum / mean / max / min of several broadcastable tensors."""
    def fwd(*a):
        r = a[0]
        for t in a[1:]:
            r = G.binary("add" if op in ("sum", "mean") else op, r, t)
        if op == "mean":
            r = F.unary("scale", r, 1.0 / len(a))
        return r, (a, r)

    def bwd(ctx, d):
        a, r = ctx
        out = []
        for t in a:
            if op in ("sum", "mean"):
                g = d if op == "sum" else F.unary("scale", d, 1.0 / len(a))
            else:  # every input equal to the result gets the gradient (reference PartialGrad)
                g = G.binary("mul", d, G.binary("eq", t, r, out_dtype=d.dtype))
            out.append(G.sum_to(g, t.shape))
        return tuple(out)
    return Fn(fwd, bwd, onnx=spec)(*xs)


def sum(*xs):  # noqa: A001
    return _nary(xs, "sum", _ox("Sum", n_in=len(xs)))


def mean(*xs):
    return _nary(xs, "mean", _ox("Mean", n_in=len(xs)))


def max(*xs):  # noqa: A001
    return _nary(xs, "max", _ox("Max", n_in=len(xs)))


def min(*xs):  # noqa: A001
    return _nary(xs, "min", _ox("Min", n_in=len(xs)))


class _Math(_Unary):
    """Native elementwise math (functional.UNARY) with an ONNX name."""
    onnx_op = ""

    @property
    def onnx(self):
        return _ox(self.onnx_op)


def _math(kind_, needs_, onnx_op):
    return type(onnx_op, (_Math,), {"kind": kind_, "needs": needs_, "onnx_op": onnx_op})


Erf, Cos, Sin, Tan = _math("erf", "x", "Erf"), _math("cos", "x", "Cos"), _math("sin", "x", "Sin"), \
    _math("tan", "y", "Tan")
Cosh, Sinh, Acos, Asin = _math("cosh", "x", "Cosh"), _math("sinh", "x", "Sinh"), _math("acos", "x", "Acos"), \
    _math("asin", "x", "Asin")
Atan, Acosh, Asinh, Atanh = _math("atan", "x", "Atan"), _math("acosh", "x", "Acosh"), _math("asinh", "x", "Asinh"), \
    _math("atanh", "x", "Atanh")
Ceil, Floor, Round, Softsign = _math("ceil", "", "Ceil"), _math("floor", "", "Floor"), _math("round", "", "Round"), \
    _math("softsign", "x", "Softsign")


def erf(x):
    return Erf()(x)


def cos(x):
    return Cos()(x)


def sin(x):
    return Sin()(x)


def tan(x):
    return Tan()(x)


def cosh(x):
    return Cosh()(x)


def sinh(x):
    return Sinh()(x)


def acos(x):
    return Acos()(x)


def asin(x):
    return Asin()(x)


def atan(x):
    return Atan()(x)


def acosh(x):
    return Acosh()(x)


def asinh(x):
    return Asinh()(x)


def atanh(x):
    return Atanh()(x)


def ceil(x):
    return Ceil()(x)


def floor(x):
    return Floor()(x)


def round(x):  # noqa: A001
    return Round()(x)


def softsign(x):
    return Softsign()(x)


def hardsigmoid(x, alpha=0.2, gamma=0.5):
    return Fn(lambda a: (G.clamp_affine(a, alpha, gamma, 0.0, 1.0), a),
              lambda a, d: G.clamp_affine(a, alpha, gamma, 0.0, 1.0, dy=d),
              onnx=_ox("HardSigmoid", {"alpha": float(alpha), "beta": float(gamma)}))(x)


def prelu(x, slope):
    def fwd(a, s):
        pos = F.unary("relu", a)
        neg = G.binary("sub", a, pos)  # min(a, 0)
        return G.binary("add", pos, G.binary("mul", neg, s)), (a, s, neg)

    def bwd(ctx, d):
        a, s, neg = ctx
        pos_mask = G.binary("gt", a, 0.0)
        # dx = d * (a > 0 ? 1 : s) = d * (mask + (1 - mask) * s)
        one_minus = G.binary("sub", G.full((), 1.0, pos_mask.dtype, pos_mask.device), pos_mask)
        coef = G.binary("add", pos_mask, G.binary("mul", one_minus, s))
        dx = G.binary("mul", d, coef)
        ds = G.sum_to(G.binary("mul", d, neg), s.shape)
        return dx, ds
    return Fn(fwd, bwd, onnx=_ox("PRelu", n_in=2))(x, slope)


def _cmp_op(op):
    def f(x, y):
        yy = y.data if isinstance(y, Tensor) else y
        return Tensor(device=x.device, data=G.binary(op, x.data, yy, out_dtype=x.dtype if x.data.is_floating_point()
                                                     else torch.float32), requires_grad=False)
    return f


less = _cmp_op("lt")
greater = _cmp_op("gt")
equal = _cmp_op("eq")
_and = _cmp_op("and")
_or = _cmp_op("or")
_xor = _cmp_op("xor")


def _not(x):
    return Tensor(device=x.device, data=G.binary("eq", x.data, 0.0), requires_grad=False)


def shape(x):
    return Tensor(device=x.device, data=torch.tensor(list(x.shape), dtype=torch.int64), requires_grad=False)


def constant_of_shape(x, value=0.0):
    shp = [int(v) for v in x.data.reshape(-1).tolist()]
    return Tensor(device=x.device, data=G.full(shp, value, torch.float32, x.data.device), requires_grad=False)


def onehot(axis, indices, depth, values):
    idx = indices.data
    vals = values.data.reshape(-1)
    off, on = float(vals[0]), float(vals[1])
    dev = idx.device
    shp = tuple(idx.shape) + (depth,)
    oh = G.full(shp, off, torch.float32, dev)
    ii = G.to(idx, torch.int64)  # negative ids wrap like numpy (ONNX OneHot)
    oh = G.scatter_elements(oh, -1, G.reshape(ii, tuple(idx.shape) + (1,)), G.full(tuple(idx.shape) + (1,), on,
                                                                                     torch.float32, dev))
    if axis != -1:
        oh = G.contiguous(oh.movedim(-1, axis))
    return Tensor(device=indices.device, data=oh, requires_grad=False)


def upsample(x, mode, scales):
    sc = [int(_b.round(float(s))) for s in scales]
    if mode != "nearest" or any(_b.abs(float(s) - r) > 1e-6 for s, r in zip(scales, sc)):
        raise NotImplementedError("upsample: nearest mode with integer scales")

    def fwd(a):
        inter = []
        src = []
        for s, r in zip(a.shape, sc):
            inter += [s, r]
            src += [s, 1]
        out = _mem.empty(inter, dtype=a.dtype, device=a.device)
        G.copy_(out, a.reshape(src).expand(*inter))
        return out.reshape([s * r for s, r in zip(a.shape, sc)]), tuple(a.shape)

    def bwd(shp, d):
        inter = []
        for s, r in zip(shp, sc):
            inter += [s, r]
        return G.reduce(G.reshape(d, inter), [2 * k + 1 for k in range(len(shp))], "sum", out_dtype=d.dtype)
    return Fn(fwd, bwd, onnx=_ox("Resize", {"mode": "nearest"}, [("in", 0), ("const", np.zeros(0, np.float32)),
                                                                 ("const", np.asarray(scales, np.float32))]))(x)


def _space_perm(x, perm, mid, out_shape, spec):
    """reshape(mid) -> permute(perm) -> reshape(out) (one native copy) and its inverse."""
    inv = tuple(int(i) for i in np.argsort(perm))
    in_shape = tuple(x.shape)
    pshape = [mid[i] for i in perm]

    def fwd(a):
        return G.reshape(G.contiguous(G.reshape(a, mid).permute(*perm)), out_shape), None

    def bwd(c, d):
        return G.reshape(G.contiguous(G.reshape(d, pshape).permute(*inv)), in_shape)
    return Fn(fwd, bwd, onnx=spec)(x)


def depth_to_space(x, blocksize, mode="DCR"):
    Nn, C, H, W = x.shape
    b = blocksize
    c = C // (b * b)
    if mode == "DCR":
        mid, perm = (Nn, b, b, c, H, W), (0, 3, 4, 1, 5, 2)
    else:  # CRD
        mid, perm = (Nn, c, b, b, H, W), (0, 1, 4, 2, 5, 3)
    return _space_perm(x, perm, mid, (Nn, c, H * b, W * b),
                       _ox("DepthToSpace", {"blocksize": blocksize, "mode": mode}))


def space_to_depth(x, blocksize, mode="DCR"):
    Nn, C, H, W = x.shape
    b = blocksize
    return _space_perm(x, (0, 3, 5, 1, 2, 4), (Nn, C, H // b, b, W // b, b), (Nn, C * b * b, H // b, W // b),
                       _ox("SpaceToDepth", {"blocksize": blocksize}))


class Embedding(Operator):
    """y = W[idx] (row gather, native index_select).  Backward scatter-adds
    the dy rows into dW (native index_add, fp32 atomics) -- no sort / unique
    / host sync, so a step using it can be captured into a HIP graph.
    Deterministic mode keeps an ordered backward (CPU reference order)."""

    def forward(self, W, idx):
        if self.requires_grad:
            self.idx, self.wshape, self.wdt = idx, W.shape, W.dtype
        return G.index_select(W, 0, idx)

    def backward(self, dy):
        i = self.idx.reshape(-1)
        self.idx = None
        d = G.reshape(dy, (-1, dy.shape[-1]))
        tgt = self.grad_target(0)
        if tgt is not None and tgt.dim() == 2 and tgt.dtype == torch.float32 and tgt.is_contiguous():
            G.index_add_(tgt, 0, i, d)
            return ACCUMULATED, None
        dw = G.zeros(self.wshape, torch.float32, dy.device)
        G.index_add_(dw, 0, i, d)
        return dw, None


def embedding(x_idx, W):
    return Embedding()(W, x_idx)


def globalaveragepool(x, keepdims=True):
    return GlobalAveragePool(keepdims)(x)


def scatter_elements(x, indices, updates, axis=0):
    idx = indices.data.long() if indices.data.dtype not in (torch.int32, torch.int64) else indices.data
    spec = _ox("ScatterElements", {"axis": axis}, [("in", 0), ("const", idx.cpu().numpy()), ("in", 1)]) \
        if _TRACE else None

    def fwd(a, u):
        ii = idx.to(a.device) if idx.device != a.device else idx
        return G.scatter_elements(a, axis, ii, u), ii

    def bwd(ii, d):
        dx = G.scatter_elements(d, axis, ii, G.zeros(ii.shape, d.dtype, d.device))
        return dx, G.gather_elements(d, axis, ii)
    return Fn(fwd, bwd, onnx=spec)(x, updates)


class Gemm(Operator):
    """ONNX/SINGA Gemm: y = alpha * op(A) op(B) + beta * C (C broadcast over
    rows); op = transpose when transA / transB.  Both products of the
    backward run on the MFMA GEMM kernels like the forward."""

    def __init__(self, alpha=1.0, beta=1.0, transA=0, transB=0, name=None):
        super().__init__(name)
        self.alpha, self.beta, self.ta, self.tb = float(alpha), float(beta), bool(transA), bool(transB)

    def forward(self, a, b, c=None):
        bias = None
        ncol = b.shape[0] if self.tb else b.shape[1]
        if c is not None and c.dim() <= 1 and c.numel() == ncol and self.beta == 1.0:
            bias = c.reshape(-1)  # row bias in the epilogue
        y = F.gemm(a, b, self.ta, self.tb, out_dtype=a.dtype, alpha=self.alpha, bias=bias)
        if c is not None and bias is None:
            y = G.binary("add", y, G.binary("mul", c, self.beta, out_dtype=y.dtype) if self.beta != 1.0 else c,
                         out_dtype=y.dtype)
        if self.requires_grad:
            self.a, self.b = a, b
            self.cshape = c.shape if c is not None else None
        return y

    def backward(self, dy):
        a, b = self.a, self.b
        self.a = self.b = None
        dy = dy.contiguous()
        da = db = None
        if self.needs_grad(0):  # d op(A) = alpha dy op(B)^T
            da = (F.gemm(b, dy, self.tb, True, out_dtype=a.dtype, alpha=self.alpha) if self.ta else
                  F.gemm(dy, b, False, not self.tb, out_dtype=a.dtype, alpha=self.alpha))
        if self.needs_grad(1):  # d op(B) = alpha op(A)^T dy
            db = (F.gemm(dy, a, True, self.ta, out_dtype=b.dtype, alpha=self.alpha) if self.tb else
                  F.gemm(a, dy, not self.ta, False, out_dtype=b.dtype, alpha=self.alpha))
        if self.cshape is None:
            return da, db
        dc = _unbroadcast(F.unary("scale", dy, self.beta) if self.beta != 1.0 else dy, self.cshape)
        return da, db, dc


def gemm(A, B, C=None, alpha=1.0, beta=1.0, transA=0, transB=0):
    op = Gemm(alpha, beta, transA, transB)
    return op(A, B, C) if C is not None else op(A, B)


def conv2d(x, W, b=None, stride=(1, 1), padding=(0, 0), dilation=(1, 1), group=1):
    op = Conv2d(stride, padding, dilation, group, has_bias=b is not None)
    return op(x, W, b) if b is not None else op(x, W)


def batchnorm_2d(x, gamma, beta, running_mean, running_var, momentum=0.1, eps=1e-5):
    return BatchNorm2d(running_mean.data if isinstance(running_mean, Tensor) else running_mean,
                       running_var.data if isinstance(running_var, Tensor) else running_var, momentum, eps)(
        x, gamma, beta)


def pooling_2d(x, kernel, stride, padding=(0, 0), is_max=True):
    return Pooling2d(kernel, stride, padding, is_max)(x)
