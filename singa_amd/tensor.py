"""``singa_amd.tensor`` -- SINGA's Tensor API over device-resident storage.

A :class:`Tensor` wraps one ``torch.Tensor`` (the storage, allocated by the
HIP caching allocator on a RocmGPU or in host memory on CppCPU) plus the
autograd bookkeeping SINGA keeps on tensors (``requires_grad``,
``stores_grad``, ``creator``).  It replaces the reference's ``Blob`` /
``SyncedMemory`` (C10, include/utils/blob.h:64-163): instead of lazy
head-state host/device syncing, tensors live on one device and move
explicitly with :meth:`Tensor.to_device` / :meth:`Tensor.to_host`.

Arithmetic on Tensors here is not recorded by autograd (as in SINGA); use
:mod:`singa_amd.autograd` operators for differentiable computation.
4-D activations on a RocmGPU may be channels_last in memory; the logical
shape is always NCHW.
"""
from __future__ import annotations

from typing import Iterable, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import device as _dev

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
            self.data = torch.zeros(tuple(int(s) for s in shape), dtype=dtype, device=self.device.torch_device)
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
        return self._wrap(self.data.contiguous())

    def _wrap(self, d: torch.Tensor, **kw) -> "Tensor":
        return Tensor(device=self.device, data=d, requires_grad=kw.get("requires_grad", self.requires_grad),
                      stores_grad=False)

    def reshape(self, shape: Sequence[int]) -> "Tensor":
        return self._wrap(self.data.reshape(tuple(shape)))

    def transpose(self, axes: Optional[Sequence[int]] = None) -> "Tensor":
        if axes is None:
            axes = tuple(reversed(range(self.data.dim())))
        return self._wrap(self.data.permute(*axes))

    def T(self) -> "Tensor":
        return self.transpose()

    def reset_like(self, t: "Tensor") -> None:
        self.data = torch.empty_like(t.data)
        self.device = t.device

    def as_type(self, dtype) -> "Tensor":
        return self._wrap(self.data.to(dtype))

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
        return float(self.data.float().abs().mean())

    def l2(self) -> float:
        return float(self.data.float().norm() / max(1, self.data.numel()) ** 0.5)

    def set_value(self, x, inplace: bool = True) -> "Tensor":
        if inplace:
            self.data.fill_(x)
            return self
        return self._wrap(torch.full_like(self.data, x))

    def copy_data(self, t: "Tensor") -> None:
        self.data.copy_(t.data.reshape(self.data.shape))

    def copy_from_numpy(self, np_array: np.ndarray, offset: int = 0) -> None:
        src = torch.from_numpy(np.ascontiguousarray(np_array))
        if offset == 0 and src.numel() == self.data.numel():
            self.data.copy_(src.reshape(self.data.shape), non_blocking=False)
        else:
            self.data.view(-1)[offset:offset + src.numel()].copy_(src.reshape(-1))

    def clone(self) -> "Tensor":
        t = self._wrap(self.data.clone())
        t.requires_grad, t.stores_grad, t.name = self.requires_grad, self.stores_grad, self.name
        return t

    def deepcopy(self) -> "Tensor":
        return self.clone()

    def copy(self) -> "Tensor":
        return self._wrap(self.data)

    def repeat(self, repeats, axis=None) -> "Tensor":
        if axis is None:
            return self._wrap(self.data.reshape(-1).repeat_interleave(repeats))
        return self._wrap(self.data.repeat_interleave(repeats, dim=axis))

    # ----------------------------------------------------------- initialisers
    def bernoulli(self, p: float, inplace: bool = True) -> "Tensor":
        d = torch.bernoulli(torch.full_like(self.data, p, dtype=torch.float32), generator=self.device.generator)
        if inplace:
            self.data.copy_(d)
            return self
        return self._wrap(d.to(self.dtype))

    def gaussian(self, mean: float, std: float, inplace: bool = True) -> "Tensor":
        d = torch.empty(self.data.shape, dtype=torch.float32, device=self.data.device)
        d.normal_(mean, std, generator=self.device.generator)
        if inplace:
            self.data.copy_(d)
            return self
        return self._wrap(d.to(self.dtype))

    def uniform(self, low: float, high: float, inplace: bool = True) -> "Tensor":
        d = torch.empty(self.data.shape, dtype=torch.float32, device=self.data.device)
        d.uniform_(low, high, generator=self.device.generator)
        if inplace:
            self.data.copy_(d)
            return self
        return self._wrap(d.to(self.dtype))

    # ------------------------------------------------- row/column broadcasts
    def add_column(self, v: "Tensor") -> None:
        self.data += v.data.reshape(-1, 1)

    def add_row(self, v: "Tensor") -> None:
        self.data += v.data.reshape(1, -1)

    def sub_column(self, v: "Tensor") -> None:
        self.data -= v.data.reshape(-1, 1)

    def sub_row(self, v: "Tensor") -> None:
        self.data -= v.data.reshape(1, -1)

    def mult_column(self, v: "Tensor") -> None:
        self.data *= v.data.reshape(-1, 1)

    def mult_row(self, v: "Tensor") -> None:
        self.data *= v.data.reshape(1, -1)

    def div_column(self, v: "Tensor") -> None:
        self.data /= v.data.reshape(-1, 1)

    def div_row(self, v: "Tensor") -> None:
        self.data /= v.data.reshape(1, -1)

    # ---------------------------------------------------------- operators
    @staticmethod
    def _raw(x):
        return x.data if isinstance(x, Tensor) else x

    def _bin(self, other, fn):
        return self._wrap(fn(self.data, self._raw(other)), requires_grad=False)

    def __add__(self, o): return self._bin(o, torch.add)
    def __radd__(self, o): return self._bin(o, lambda a, b: b + a)
    def __sub__(self, o): return self._bin(o, torch.sub)
    def __rsub__(self, o): return self._bin(o, lambda a, b: b - a)
    def __mul__(self, o): return self._bin(o, torch.mul)
    def __rmul__(self, o): return self._bin(o, lambda a, b: b * a)
    def __truediv__(self, o): return self._bin(o, torch.div)
    def __rtruediv__(self, o): return self._bin(o, lambda a, b: b / a)
    def __matmul__(self, o): return self._bin(o, torch.matmul)
    def __pow__(self, o): return self._bin(o, torch.pow)
    def __lt__(self, o): return self._bin(o, lambda a, b: (a < b).to(self.dtype))
    def __le__(self, o): return self._bin(o, lambda a, b: (a <= b).to(self.dtype))
    def __gt__(self, o): return self._bin(o, lambda a, b: (a > b).to(self.dtype))
    def __ge__(self, o): return self._bin(o, lambda a, b: (a >= b).to(self.dtype))
    def __neg__(self): return self._wrap(-self.data, requires_grad=False)
    def __abs__(self): return self._wrap(self.data.abs(), requires_grad=False)

    def __iadd__(self, o):
        self.data += self._raw(o)
        return self

    def __isub__(self, o):
        self.data -= self._raw(o)
        return self

    def __imul__(self, o):
        self.data *= self._raw(o)
        return self

    def __itruediv__(self, o):
        self.data /= self._raw(o)
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


def to_numpy(t: Tensor) -> np.ndarray:
    d = t.data.detach()
    if d.dtype == torch.bfloat16:
        d = d.float()
    return d.cpu().contiguous().numpy()


def to_raw(t) -> torch.Tensor:
    return t.data if isinstance(t, Tensor) else t


def zeros(shape, dev=None, dtype=float32) -> Tensor:
    return Tensor(shape, dev, dtype)


def ones(shape, dev=None, dtype=float32) -> Tensor:
    t = Tensor(shape, dev, dtype)
    t.data.fill_(1)
    return t


def zeros_like(t: Tensor) -> Tensor:
    return Tensor(device=t.device, data=torch.zeros_like(t.data))


def ones_like(t: Tensor) -> Tensor:
    return Tensor(device=t.device, data=torch.ones_like(t.data))


def random(shape, dev=None) -> Tensor:
    t = Tensor(shape, dev)
    return t.uniform(0.0, 1.0)


def product(shape) -> int:
    r = 1
    for s in shape:
        r *= int(s)
    return r


def sizeof(dtype) -> int:
    return torch.empty((), dtype=dtype).element_size()


def reshape(t: Tensor, shape) -> Tensor:
    return t.reshape(shape)


def transpose(t: Tensor, axes=None) -> Tensor:
    return t.transpose(axes)


def copy_data_to_from(dst: Tensor, src: Tensor, size: int, dst_offset: int = 0, src_offset: int = 0) -> None:
    dst.data.view(-1)[dst_offset:dst_offset + size].copy_(src.data.reshape(-1)[src_offset:src_offset + size])


def _u(fn):
    def f(t: Tensor) -> Tensor:
        return Tensor(device=t.device, data=fn(t.data), requires_grad=False)
    return f


abs = _u(torch.abs)  # noqa: A001
exp = _u(torch.exp)
log = _u(torch.log)
sigmoid = _u(torch.sigmoid)
sign = _u(torch.sign)
sqrt = _u(torch.sqrt)
square = _u(torch.square)
tanh = _u(torch.tanh)
relu = _u(torch.relu)
ceil = _u(torch.ceil)
floor = _u(torch.floor)
round = _u(torch.round)  # noqa: A001
cos = _u(torch.cos)
sin = _u(torch.sin)
tan = _u(torch.tan)
acos = _u(torch.acos)
asin = _u(torch.asin)
atan = _u(torch.atan)
cosh = _u(torch.cosh)
sinh = _u(torch.sinh)
erf = _u(torch.erf)


def sum(t: Tensor, axis=None, keepdims: bool = False) -> Union[Tensor, float]:  # noqa: A001
    if axis is None:
        return float(t.data.float().sum())
    return Tensor(device=t.device, data=t.data.sum(dim=axis, keepdim=keepdims), requires_grad=False)


def average(t: Tensor, axis=None) -> Union[Tensor, float]:
    if axis is None:
        return float(t.data.float().mean())
    return Tensor(device=t.device, data=t.data.float().mean(dim=axis).to(t.dtype), requires_grad=False)


def pow(t: Tensor, x, out=None) -> Tensor:  # noqa: A001
    r = torch.pow(t.data, Tensor._raw(x))
    if out is not None:
        out.data.copy_(r)
        return out
    return Tensor(device=t.device, data=r, requires_grad=False)


def softmax(t: Tensor, out=None, axis: int = -1) -> Tensor:
    from .ops import functional as F

    r = F.softmax(t.data, axis)
    if out is not None:
        out.data.copy_(r)
        return out
    return Tensor(device=t.device, data=r, requires_grad=False)


def _cmp(fn):
    def f(t: Tensor, x) -> Tensor:
        return Tensor(device=t.device, data=fn(t.data, Tensor._raw(x)).to(t.dtype), requires_grad=False)
    return f


lt = _cmp(torch.lt)
le = _cmp(torch.le)
gt = _cmp(torch.gt)
ge = _cmp(torch.ge)
eq = _cmp(torch.eq)


def add(lhs, rhs, ret=None):
    r = Tensor._raw(lhs) + Tensor._raw(rhs)
    if ret is not None:
        ret.data.copy_(r)
        return ret
    return Tensor(device=lhs.device, data=r, requires_grad=False)


def sub(lhs, rhs, ret=None):
    r = Tensor._raw(lhs) - Tensor._raw(rhs)
    if ret is not None:
        ret.data.copy_(r)
        return ret
    return Tensor(device=lhs.device, data=r, requires_grad=False)


def eltwise_mult(lhs, rhs, ret=None):
    r = Tensor._raw(lhs) * Tensor._raw(rhs)
    if ret is not None:
        ret.data.copy_(r)
        return ret
    return Tensor(device=lhs.device, data=r, requires_grad=False)


def div(lhs, rhs, ret=None):
    r = Tensor._raw(lhs) / Tensor._raw(rhs)
    if ret is not None:
        ret.data.copy_(r)
        return ret
    return Tensor(device=lhs.device, data=r, requires_grad=False)


def mult(A: Tensor, B: Tensor, C: Optional[Tensor] = None, alpha: float = 1.0, beta: float = 0.0) -> Tensor:
    """C = alpha*A@B + beta*C (matrix product, as singa.tensor.mult)."""
    r = alpha * torch.matmul(A.data, B.data)
    if C is None:
        return Tensor(device=A.device, data=r, requires_grad=False)
    C.data.mul_(beta).add_(r)
    return C


def axpy(alpha: float, x: Tensor, y: Tensor) -> Tensor:
    y.data.add_(x.data, alpha=alpha)
    return y


def bernoulli(p: float, t: Tensor) -> Tensor:
    return t.bernoulli(p)


def gaussian(mean: float, std: float, t: Tensor) -> Tensor:
    return t.gaussian(mean, std)


def uniform(low: float, high: float, t: Tensor) -> Tensor:
    return t.uniform(low, high)


def add_column(alpha, v, beta, M):
    M.data.mul_(beta).add_(alpha * v.data.reshape(-1, 1))
    return M


def add_row(alpha, v, beta, M):
    M.data.mul_(beta).add_(alpha * v.data.reshape(1, -1))
    return M


def sum_columns(M: Tensor) -> Tensor:
    return Tensor(device=M.device, data=M.data.sum(dim=1), requires_grad=False)


def sum_rows(M: Tensor) -> Tensor:
    return Tensor(device=M.device, data=M.data.sum(dim=0), requires_grad=False)


def concatenate(tensors: Sequence[Tensor], axis: int) -> Tensor:
    return Tensor(device=tensors[0].device, data=torch.cat([t.data for t in tensors], dim=axis),
                  requires_grad=False)


def einsum(ops: str, *args: Tensor) -> Tensor:
    return Tensor(device=args[0].device, data=torch.einsum(ops, *[a.data for a in args]), requires_grad=False)


def tensordot(A: Tensor, B: Tensor, axes=2) -> Tensor:
    return Tensor(device=A.device, data=torch.tensordot(A.data, B.data, dims=axes), requires_grad=False)


def repeat(t: Tensor, repeats, axis=None) -> Tensor:
    return t.repeat(repeats, axis)


def get_dtype(t: Tensor):
    return t.dtype
