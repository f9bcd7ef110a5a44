"""``singa_amd.tensor`` -- SINGA's Tensor API over device-resident storage.

A :class:`Tensor` wraps one ``torch.Tensor`` (the storage, allocated by the
HIP caching allocator on a RocmGPU or in host memory on CppCPU) plus the
autograd bookkeeping SINGA keeps on tensors (``requires_grad``,
``stores_grad``, ``creator``).  It replaces the reference's ``Blob`` /
``SyncedMemory`` (C10, include/utils/blob.h:64-163): instead of lazy
head-state host/device syncing, tensors live on one device and move
explicitly with :meth:`Tensor.to_device` / :meth:`Tensor.to_host`.

Arithmetic on Tensors here is not recorded by autograd (as in SINGA); use
:mod:`singa_amd.autograd` operators for differentiable computation.  Every
math / layout / init op dispatches through :mod:`singa_amd.ops.glue` and
:mod:`singa_amd.ops.functional`: a hand-written gfx950 kernel on a RocmGPU,
the host reference on CppCPU.
4-D activations on a RocmGPU may be channels_last in memory; the logical
shape is always NCHW.
"""
from __future__ import annotations

from typing import Iterable, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import memory as _mem
from . import device as _dev
from .ops import functional as _F
from .ops import glue as _G

float16 = torch.float16
float32 = torch.float32
bfloat16 = torch.bfloat16
int32 = torch.int32
int64 = torch.int64
uint8 = torch.uint8
bool_ = torch.bool

_NP2T = {np.dtype(np.float32): torch.float32, np.dtype(np.float16): torch.float16, np.dtype(np.int32): torch.int32,
         np.dtype(np.int64): torch.int64, np.dtype(np.uint8): torch.uint8, np.dtype(np.float64): torch.float32,
         np.dtype(np.bool_): torch.bool}


def _dev_of(device) -> _dev.Device:
    return device if device is not None else _dev.get_default_device()


class Tensor:
    """SINGA tensor.  ``data`` is the backing ``torch.Tensor``."""

    __slots__ = ("data", "device", "requires_grad", "stores_grad", "creator", "name", "_grad", "__weakref__",
                 "grad_view", "low", "param_meta", "_host_np")

    def __init__(self, shape: Sequence[int] = (), device: Optional[_dev.Device] = None, dtype=float32,
                 data=None, requires_grad: bool = True, stores_grad: bool = False, creator=None,
                 name: Optional[str] = None):
        self.device = _dev_of(device)
        if data is not None:
            if isinstance(data, Tensor):
                data = data.data
            if isinstance(data, np.ndarray):
                data = torch.from_numpy(np.ascontiguousarray(data))
            if not isinstance(data, torch.Tensor):
                data = torch.as_tensor(data)
            if data.device != self.device.torch_device:
                data = data.to(self.device.torch_device)
            self.data = data
        else:
            self.data = _G.zeros(tuple(int(s) for s in shape), dtype, self.device.torch_device)
        self.requires_grad = requires_grad
        self.stores_grad = stores_grad
        self.creator = creator
        self.name = name
        self._grad = None
        self.grad_view = None   # fp32 view into a flat gradient buffer (set by ParamStore)
        self.low = None         # bf16 compute copy (mixed precision), view into flat buffer
        self.param_meta = None  # dict: lr_mult, wd_mult, ...

    # ------------------------------------------------------------------ basics
    @property
    def shape(self) -> Tuple[int, ...]:
        return tuple(self.data.shape)

    @property
    def dtype(self):
        return self.data.dtype

    @property
    def grad(self):
        return self._grad

    @grad.setter
    def grad(self, g):
        self._grad = g

    def ndim(self) -> int:
        return self.data.dim()

    def is_empty(self) -> bool:
        return self.data.numel() == 0

    def is_transpose(self) -> bool:
        return not self.data.is_contiguous() and not (self.data.dim() == 4 and self.data.is_contiguous(
            memory_format=torch.channels_last))

    def size(self) -> int:
        return self.data.numel()

    def memsize(self) -> int:
        return self.data.numel() * self.data.element_size()

    def __len__(self):
        return self.data.shape[0] if self.data.dim() else 1

    def contiguous(self) -> "Tensor":
        return self._wrap(_G.contiguous(self.data))

    def _wrap(self, d: torch.Tensor, **kw) -> "Tensor":
        return Tensor(device=self.device, data=d, requires_grad=kw.get("requires_grad", self.requires_grad),
                      stores_grad=False)

    @property
    def native(self):
        """The framework-owned handle of this tensor's bytes (``_C.mem.Tensor``:
        storage, offset, shape, strides, dtype, device; native views and
        DLPack export -- see :func:`singa_amd.memory.native`)."""
        return _mem.native(self.data)

    @classmethod
    def from_native(cls, h, device: Optional[_dev.Device] = None, requires_grad: bool = True) -> "Tensor":
        """Wrap a native handle (no copy)."""
        return cls(device=device, data=_mem.to_torch(h), requires_grad=requires_grad)

    def _native_ok(self) -> bool:
        return _mem.native_views() and self.data.dtype in _mem._CODES and self.data.numel() > 0

    def reshape(self, shape: Sequence[int]) -> "Tensor":
        # a native view over the same storage when the layout allows, else a copy
        if self._native_ok() and self.data.is_contiguous():
            return self._wrap(_mem.to_torch(_mem.native(self.data).reshape([int(v) for v in shape])))
        return self._wrap(_G.reshape(self.data, tuple(shape)))

    def transpose(self, axes: Optional[Sequence[int]] = None) -> "Tensor":
        if axes is None:
            axes = tuple(reversed(range(self.data.dim())))
        if self._native_ok():
            return self._wrap(_mem.to_torch(_mem.native(self.data).permute([int(a) for a in axes])))
        return self._wrap(self.data.permute(*axes))

    def T(self) -> "Tensor":
        return self.transpose()

    def reset_like(self, t: "Tensor") -> None:
        self.data = _mem.empty_like(t.data)
        self.device = t.device

    def as_type(self, dtype) -> "Tensor":
        return self._wrap(_G.to(self.data, dtype))

    to_type = as_type

    def to_device(self, device: _dev.Device) -> "Tensor":
        """In-place move (SINGA semantics); returns self."""
        if device.torch_device != self.data.device:
            self.data = self.data.to(device.torch_device)
        self.device = device
        return self

    def to_host(self) -> "Tensor":
        return self.to_device(_dev.create_cpu_device())

    def l1(self) -> float:
        return float(_G.reduce(_F.unary("abs", _G.to(self.data, _f32(self.data))), None, "mean",
                               out_dtype=torch.float32))

    def l2(self) -> float:
        ss = float(_G.reduce(_G.to(self.data, _f32(self.data)), None, "sumsq", out_dtype=torch.float32))
        return (ss / max(1, self.data.numel())) ** 0.5

    def set_value(self, x, inplace: bool = True) -> "Tensor":
        if inplace:
            _G.fill_(self.data, x)
            return self
        return self._wrap(_G.full(self.data.shape, x, self.data.dtype, self.data.device))

    def copy_data(self, t: "Tensor") -> None:
        _G.copy_(self.data, _G.reshape(t.data, self.data.shape))

    def copy_from_numpy(self, np_array: np.ndarray, offset: int = 0) -> None:
        src = torch.from_numpy(np.ascontiguousarray(np_array))
        if offset == 0 and src.numel() == self.data.numel():
            _G.copy_(self.data, src.reshape(self.data.shape))
        else:
            _G.copy_(self.data.view(-1)[offset:offset + src.numel()], src.reshape(-1))

    def clone(self) -> "Tensor":
        t = self._wrap(_G.copy_(_mem.empty(self.data.shape, dtype=self.data.dtype, device=self.data.device),
                                self.data))
        t.requires_grad, t.stores_grad, t.name = self.requires_grad, self.stores_grad, self.name
        return t

    def deepcopy(self) -> "Tensor":
        return self.clone()

    def copy(self) -> "Tensor":
        return self._wrap(self.data)

    def repeat(self, repeats, axis=None) -> "Tensor":
        d = self.data.reshape(-1) if axis is None else self.data
        ax = 0 if axis is None else axis % d.dim()
        v = d.unsqueeze(ax + 1)
        shape = list(v.shape)
        shape[ax + 1] = int(repeats)
        out = _G.contiguous(v.expand(*shape))
        shape[ax] *= int(repeats)
        del shape[ax + 1]
        return self._wrap(out.reshape(shape))

    # ----------------------------------------------------------- initialisers
    def bernoulli(self, p: float, inplace: bool = True) -> "Tensor":
        u = _G.random_(_mem.empty(self.data.shape, dtype=torch.float32, device=self.data.device), "uniform", 0.0,
                       1.0, self.device)
        d = _G.binary("lt", u, float(p))
        if inplace:
            _G.copy_(self.data, d)
            return self
        return self._wrap(_G.to(d, self.dtype))

    def gaussian(self, mean: float, std: float, inplace: bool = True) -> "Tensor":
        d = self.data if inplace else _mem.empty(self.data.shape, dtype=self.dtype, device=self.data.device)
        _G.random_(d, "gaussian", mean, std, self.device)
        return self if inplace else self._wrap(d)

    def uniform(self, low: float, high: float, inplace: bool = True) -> "Tensor":
        d = self.data if inplace else _mem.empty(self.data.shape, dtype=self.dtype, device=self.data.device)
        _G.random_(d, "uniform", low, high, self.device)
        return self if inplace else self._wrap(d)

    # ------------------------------------------------- row/column broadcasts
    def _ibin(self, op: str, v) -> None:
        _G.binary(op, self.data, self._raw(v), out=self.data)

    def add_column(self, v: "Tensor") -> None:
        self._ibin("add", v.data.reshape(-1, 1))

    def add_row(self, v: "Tensor") -> None:
        self._ibin("add", v.data.reshape(1, -1))

    def sub_column(self, v: "Tensor") -> None:
        self._ibin("sub", v.data.reshape(-1, 1))

    def sub_row(self, v: "Tensor") -> None:
        self._ibin("sub", v.data.reshape(1, -1))

    def mult_column(self, v: "Tensor") -> None:
        self._ibin("mul", v.data.reshape(-1, 1))

    def mult_row(self, v: "Tensor") -> None:
        self._ibin("mul", v.data.reshape(1, -1))

    def div_column(self, v: "Tensor") -> None:
        self._ibin("div", v.data.reshape(-1, 1))

    def div_row(self, v: "Tensor") -> None:
        self._ibin("div", v.data.reshape(1, -1))

    # ---------------------------------------------------------- operators
    @staticmethod
    def _raw(x):
        return x.data if isinstance(x, Tensor) else x

    def _bin(self, other, op: str, rev: bool = False, cmp: bool = False):
        a, b = self.data, self._raw(other)
        if rev:
            if not isinstance(b, torch.Tensor):
                b = _G.full((), b, a.dtype if a.is_floating_point() else torch.float32, a.device)
            a, b = b, a
        r = _G.binary(op, a, b, out_dtype=self.dtype if cmp else None)
        return self._wrap(r, requires_grad=False)

    def __add__(self, o): return self._bin(o, "add")
    def __radd__(self, o): return self._bin(o, "add", rev=True)
    def __sub__(self, o): return self._bin(o, "sub")
    def __rsub__(self, o): return self._bin(o, "sub", rev=True)
    def __mul__(self, o): return self._bin(o, "mul")
    def __rmul__(self, o): return self._bin(o, "mul", rev=True)
    def __truediv__(self, o): return self._bin(o, "div")
    def __rtruediv__(self, o): return self._bin(o, "div", rev=True)
    def __matmul__(self, o): return self._wrap(_F.matmul(self.data, self._raw(o)), requires_grad=False)
    def __pow__(self, o): return self._bin(o, "pow")
    def __lt__(self, o): return self._bin(o, "lt", cmp=True)
    def __le__(self, o): return self._bin(o, "le", cmp=True)
    def __gt__(self, o): return self._bin(o, "gt", cmp=True)
    def __ge__(self, o): return self._bin(o, "ge", cmp=True)
    def __neg__(self): return self._wrap(_F.unary("neg", self.data), requires_grad=False)
    def __abs__(self): return self._wrap(_F.unary("abs", self.data), requires_grad=False)

    def __iadd__(self, o):
        self._ibin("add", o)
        return self

    def __isub__(self, o):
        self._ibin("sub", o)
        return self

    def __imul__(self, o):
        self._ibin("mul", o)
        return self

    def __itruediv__(self, o):
        self._ibin("div", o)
        return self

    def __getitem__(self, idx):
        return self._wrap(self.data[idx])

    def __repr__(self):
        return f"Tensor(shape={self.shape}, dtype={self.dtype}, device={self.device}, name={self.name})"

    def numpy(self) -> np.ndarray:
        return to_numpy(self)


# ---------------------------------------------------------------------------
# module-level functions (singa.tensor)
# ---------------------------------------------------------------------------
def from_numpy(np_array: np.ndarray, dev: Optional[_dev.Device] = None, requires_grad: bool = False) -> Tensor:
    a = np.ascontiguousarray(np_array)
    if a.dtype == np.float64:
        a = a.astype(np.float32)
    return Tensor(device=dev or _dev.get_default_device(), data=torch.from_numpy(a), requires_grad=requires_grad)


def from_raw_tensor(t: torch.Tensor, dev: Optional[_dev.Device] = None) -> Tensor:
    return Tensor(device=dev or _dev.get_default_device(), data=t)


def _f32(d: torch.Tensor) -> torch.dtype:
    return d.dtype if d.dtype in (torch.float32, torch.bfloat16) else torch.float32


def to_numpy(t: Tensor) -> np.ndarray:
    d = t.data.detach()
    if d.dtype == torch.bfloat16:
        d = _G.to(d, torch.float32)
    return _G.contiguous(d).cpu().numpy()


def to_raw(t) -> torch.Tensor:
    return t.data if isinstance(t, Tensor) else t


def zeros(shape, dev=None, dtype=float32) -> Tensor:
    return Tensor(shape, dev, dtype)


def ones(shape, dev=None, dtype=float32) -> Tensor:
    t = Tensor(shape, dev, dtype)
    _G.fill_(t.data, 1)
    return t


def zeros_like(t: Tensor) -> Tensor:
    return Tensor(device=t.device, data=_G.zeros_like(t.data))


def ones_like(t: Tensor) -> Tensor:
    return Tensor(device=t.device, data=_G.fill_(_G.zeros_like(t.data), 1.0))


def random(shape, dev=None) -> Tensor:
    t = Tensor(shape, dev)
    return t.uniform(0.0, 1.0)


def product(shape) -> int:
    r = 1
    for s in shape:
        r *= int(s)
    return r


def sizeof(dtype) -> int:
    return _mem.empty((), dtype=dtype).element_size()


def reshape(t: Tensor, shape) -> Tensor:
    return t.reshape(shape)


def transpose(t: Tensor, axes=None) -> Tensor:
    return t.transpose(axes)


def copy_data_to_from(dst: Tensor, src: Tensor, size: int, dst_offset: int = 0, src_offset: int = 0) -> None:
    _G.copy_(dst.data.view(-1)[dst_offset:dst_offset + size], _G.reshape(src.data, (-1,))[src_offset:src_offset + size])


def _u(op):
    def f(t: Tensor) -> Tensor:
        return Tensor(device=t.device, data=_F.unary(op, t.data), requires_grad=False)
    return f


abs = _u("abs")  # noqa: A001
exp = _u("exp")
log = _u("log")
sigmoid = _u("sigmoid")
sign = _u("sign")
sqrt = _u("sqrt")
square = _u("square")
tanh = _u("tanh")
relu = _u("relu")
ceil = _u("ceil")
floor = _u("floor")
round = _u("round")  # noqa: A001
cos = _u("cos")
sin = _u("sin")
tan = _u("tan")
acos = _u("acos")
asin = _u("asin")
atan = _u("atan")
cosh = _u("cosh")
sinh = _u("sinh")
erf = _u("erf")


def sum(t: Tensor, axis=None, keepdims: bool = False) -> Union[Tensor, float]:  # noqa: A001
    if axis is None:
        return float(_G.reduce(t.data, None, "sum", out_dtype=torch.float32))
    axes = [axis] if isinstance(axis, int) else list(axis)
    return Tensor(device=t.device, data=_G.reduce(t.data, axes, "sum", keepdims), requires_grad=False)


def average(t: Tensor, axis=None) -> Union[Tensor, float]:
    if axis is None:
        return float(_G.reduce(t.data, None, "mean", out_dtype=torch.float32))
    axes = [axis] if isinstance(axis, int) else list(axis)
    return Tensor(device=t.device, data=_G.reduce(t.data, axes, "mean", out_dtype=_f32(t.data)),
                  requires_grad=False)


def _ret(r: torch.Tensor, like: Tensor, out: Optional[Tensor]) -> Tensor:
    if out is not None:
        _G.copy_(out.data, r)
        return out
    return Tensor(device=like.device, data=r, requires_grad=False)


def pow(t: Tensor, x, out=None) -> Tensor:  # noqa: A001
    return _ret(_G.binary("pow", t.data, Tensor._raw(x)), t, out)


def softmax(t: Tensor, out=None, axis: int = -1) -> Tensor:
    return _ret(_F.softmax(t.data, axis), t, out)


def _cmp(op):
    def f(t: Tensor, x) -> Tensor:
        return Tensor(device=t.device, data=_G.binary(op, t.data, Tensor._raw(x), out_dtype=_f32(t.data)),
                      requires_grad=False)
    return f


lt = _cmp("lt")
le = _cmp("le")
gt = _cmp("gt")
ge = _cmp("ge")
eq = _cmp("eq")


def add(lhs, rhs, ret=None):
    return _ret(_G.binary("add", Tensor._raw(lhs), Tensor._raw(rhs)), lhs, ret)


def sub(lhs, rhs, ret=None):
    return _ret(_G.binary("sub", Tensor._raw(lhs), Tensor._raw(rhs)), lhs, ret)


def eltwise_mult(lhs, rhs, ret=None):
    return _ret(_G.binary("mul", Tensor._raw(lhs), Tensor._raw(rhs)), lhs, ret)


def div(lhs, rhs, ret=None):
    return _ret(_G.binary("div", Tensor._raw(lhs), Tensor._raw(rhs)), lhs, ret)


def mult(A: Tensor, B: Tensor, C: Optional[Tensor] = None, alpha: float = 1.0, beta: float = 0.0) -> Tensor:
    """C = alpha*A@B + beta*C (matrix product, as singa.tensor.mult) on the
    MFMA GEMM kernels (bf16, or exact fp32)."""
    if C is None:
        return Tensor(device=A.device, data=_F.gemm(A.data, B.data, out_dtype=A.dtype, alpha=alpha),
                      requires_grad=False)
    if C.data.is_contiguous() and C.data.dtype in (torch.float32, torch.bfloat16) and A.dtype == B.dtype:
        _F.gemm(A.data, B.data, out=C.data, alpha=alpha, beta=beta)
        return C
    r = _F.gemm(A.data, B.data, out_dtype=torch.float32, alpha=alpha)
    _G.copy_(C.data, _G.binary("add", _G.binary("mul", C.data, beta, out_dtype=torch.float32), r))
    return C


def axpy(alpha: float, x: Tensor, y: Tensor) -> Tensor:
    _G.binary("add", y.data, _F.unary("scale", _G.to(x.data, y.dtype), alpha), out=y.data)
    return y


def bernoulli(p: float, t: Tensor) -> Tensor:
    return t.bernoulli(p)


def gaussian(mean: float, std: float, t: Tensor) -> Tensor:
    return t.gaussian(mean, std)


def uniform(low: float, high: float, t: Tensor) -> Tensor:
    return t.uniform(low, high)


def add_column(alpha, v, beta, M):
    _G.copy_(M.data, _G.binary("add", _G.binary("mul", M.data, beta),
                               _G.binary("mul", v.data.reshape(-1, 1), alpha)))
    return M


def add_row(alpha, v, beta, M):
    _G.copy_(M.data, _G.binary("add", _G.binary("mul", M.data, beta),
                               _G.binary("mul", v.data.reshape(1, -1), alpha)))
    return M


def sum_columns(M: Tensor) -> Tensor:
    return Tensor(device=M.device, data=_G.reduce(M.data, [1], "sum"), requires_grad=False)


def sum_rows(M: Tensor) -> Tensor:
    return Tensor(device=M.device, data=_G.reduce(M.data, [0], "sum"), requires_grad=False)


def concatenate(tensors: Sequence[Tensor], axis: int) -> Tensor:
    return Tensor(device=tensors[0].device, data=_G.cat([t.data for t in tensors], axis), requires_grad=False)


def _contract(a: torch.Tensor, la: str, b: torch.Tensor, lb: str, lo: str) -> torch.Tensor:
    """Two-operand einsum as permute -> batched GEMM -> permute (native
    copies + the MFMA GEMM on the GPU)."""
    sizes = {}
    for t, ls in ((a, la), (b, lb)):
        for c, n in zip(ls, t.shape):
            sizes[c] = n
    # labels in one operand only and absent from the output: sum them first
    for which in (0, 1):
        t, ls, other = (a, la, lb) if which == 0 else (b, lb, la)
        drop = [k for k, c in enumerate(ls) if c not in other and c not in lo]
        if drop:
            t = _G.reduce(t, drop, "sum", out_dtype=t.dtype)
            ls = "".join(c for k, c in enumerate(ls) if k not in drop)
            if which == 0:
                a, la = t, ls
            else:
                b, lb = t, ls
    batch = [c for c in la if c in lb and c in lo]
    con = [c for c in la if c in lb and c not in lo]
    ao = [c for c in la if c not in lb]
    bo = [c for c in lb if c not in la]
    prod = lambda cs: int(np.prod([sizes[c] for c in cs])) if cs else 1  # noqa: E731
    a3 = _G.reshape(_G.contiguous(a.permute(*[la.index(c) for c in batch + ao + con])),
                    (prod(batch), prod(ao), prod(con)))
    b3 = _G.reshape(_G.contiguous(b.permute(*[lb.index(c) for c in batch + con + bo])),
                    (prod(batch), prod(con), prod(bo)))
    r = _F.gemm(a3, b3, out_dtype=a.dtype)
    got = batch + ao + bo
    r = r.reshape([sizes[c] for c in got])
    return _G.contiguous(r.permute(*[got.index(c) for c in lo])) if got != list(lo) else r


def einsum(ops: str, *args: Tensor) -> Tensor:
    """einsum of one or two operands (no repeated labels within an operand)."""
    lhs, lo = ops.replace(" ", "").split("->")
    ins = lhs.split(",")
    if len(ins) == 1:
        la = ins[0]
        d = args[0].data
        drop = [k for k, c in enumerate(la) if c not in lo]
        if drop:
            d = _G.reduce(d, drop, "sum", out_dtype=d.dtype)
            la = "".join(c for k, c in enumerate(la) if k not in drop)
        r = _G.contiguous(d.permute(*[la.index(c) for c in lo])) if la != lo else d
        return Tensor(device=args[0].device, data=r, requires_grad=False)
    if len(ins) != 2:
        raise NotImplementedError("einsum: one or two operands")
    r = _contract(args[0].data, ins[0], args[1].data, ins[1], lo)
    return Tensor(device=args[0].device, data=r, requires_grad=False)


def tensordot(A: Tensor, B: Tensor, axes=2) -> Tensor:
    if isinstance(axes, int):
        ax_a = list(range(A.ndim() - axes, A.ndim()))
        ax_b = list(range(axes))
    else:
        ax_a, ax_b = [list(x) if not isinstance(x, int) else [x] for x in axes]
    letters = "abcdefghijklmnopqrstuvwxyz"
    la = letters[:A.ndim()]
    lb = [None] * B.ndim()
    for i, j in zip(ax_a, ax_b):
        lb[j] = la[i]
    extra = iter(letters[A.ndim():])
    lb = "".join(c if c is not None else next(extra) for c in lb)
    lo = "".join(c for k, c in enumerate(la) if k not in ax_a) + "".join(c for c in lb if c not in la)
    return Tensor(device=A.device, data=_contract(A.data, la, B.data, lb, lo), requires_grad=False)


def repeat(t: Tensor, repeats, axis=None) -> Tensor:
    return t.repeat(repeats, axis)


def get_dtype(t: Tensor):
    return t.dtype
