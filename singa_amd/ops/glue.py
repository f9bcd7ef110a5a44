"""Layout / indexing / broadcast / reduction ops ("glue") on raw ``torch.Tensor``
storage, dispatching to the gfx950 kernels of ``csrc/kernels/glue.hip`` on
the GPU and to the native C++ loops of ``_core.cpu`` (csrc/runtime/cpu_ops.cc)
for host tensors -- the CppCPU device.  The plain PyTorch expressions kept
below each native branch are the numerics oracle of the tests
(``cpu.torch_oracle()``) and the path of host dtypes without a kernel.

Every GPU op here runs a hand-written kernel; PyTorch supplies storage and
free *views* only (slicing, transposes, expand, reshape of contiguous data
launch nothing).  Anything that must move data -- making a view dense,
changing the memory format or dtype, concatenation, padding, gathers,
scatters, broadcasting arithmetic and reductions -- is one native launch.

Reference counterparts: the mshadow expression plans reshape / swapaxis /
pad / crop / mirror / broadcast / repmat / sum_rows / sumall_except_dim
(include/mshadow/tensor_expr_ext.h:354-577,706-912) and the connection
layers' slice / concat (src/worker/base_layer.cc:85-173).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch

from .. import memory as _mem
from . import cpu as CP
from . import native as N

BIN = {"add": 0, "sub": 1, "mul": 2, "div": 3, "pow": 4, "max": 5, "min": 6, "lt": 7, "le": 8, "gt": 9, "ge": 10,
       "eq": 11, "ne": 12, "and": 13, "or": 14, "xor": 15}
RED = {"sum": 0, "mean": 1, "max": 2, "min": 3, "sumsq": 4}
PAD = {"constant": 0, "reflect": 1, "edge": 2}
_FLOATS = (torch.float32, torch.bfloat16)


def on_gpu(*ts) -> bool:
    """True when the operands live on the GPU and the native path is on
    (native._TORCH_ORACLE_FOR_TESTS -- a test-only hook -- routes everything to PyTorch)."""
    return any(t is not None and t.is_cuda for t in ts) and N.force_native()


def _lib():
    return N.lib()


def coalesce(size: Sequence[int], *strides: Sequence[int]):
    """Drop size-1 dims and merge adjacent dims that are jointly contiguous
    in every operand; returns (size, strides_0, strides_1, ...)."""
    dims = [(s, [st[k] for st in strides]) for k, s in enumerate(size) if s != 1]
    if not dims:
        return [1], *[[0] for _ in strides]
    out = [dims[-1]]
    for s, st in reversed(dims[:-1]):
        s0, st0 = out[-1]
        if all(a == b * s0 for a, b in zip(st, st0)):
            out[-1] = (s * s0, st0)
        else:
            out.append((s, st))
    out.reverse()
    return [s for s, _ in out], *[[st[i] for _, st in out] for i in range(len(strides))]


def _bstrides(t: torch.Tensor, shape) -> List[int]:
    """Element strides of t broadcast to `shape` (0 on broadcast dims)."""
    nd = len(shape)
    st = [0] * nd
    off = nd - t.dim()
    for k in range(t.dim()):
        st[off + k] = 0 if (t.shape[k] == 1 and shape[off + k] != 1) else t.stride(k)
    return st


# ------------------------------------------------------------- host transfer
_NP_OF = {torch.float32: "float32", torch.float64: "float64", torch.float16: "float16", torch.int32: "int32",
          torch.int64: "int64", torch.int16: "int16", torch.int8: "int8", torch.uint8: "uint8", torch.bool: "bool"}


def to_numpy(t: torch.Tensor):
    """A host numpy copy of ``t`` (bf16 widened to fp32).  Device tensors
    are made dense by a native kernel and copied with one stream-ordered
    hipMemcpy (csrc/mem/stream_graph.cpp), no PyTorch copy."""
    import numpy as np

    if t.dtype == torch.bfloat16:
        t = to(t, torch.float32)
    if not t.is_cuda:
        return t.detach().contiguous().numpy().copy()
    d = contiguous(t)
    out = np.empty(tuple(d.shape), dtype=_NP_OF[d.dtype])
    if out.nbytes:
        _lib().rt.memcpy_d2h(out.ctypes.data, d.data_ptr(), out.nbytes, N.stream(d.device.index))
    return out


def from_numpy(a, device) -> torch.Tensor:
    """A dense device (or host) tensor holding numpy array ``a``, in the
    native pool; dtypes are kept (float64 included)."""
    import numpy as np

    a = np.ascontiguousarray(a)
    dev = device if isinstance(device, torch.device) else torch.device(device)
    dt = {v: k for k, v in _NP_OF.items()}[a.dtype.name]
    out = _mem.empty(tuple(a.shape), dtype=dt, device=dev)
    if dev.type != "cuda":
        out.copy_(torch.from_numpy(a))
        return out
    if a.nbytes:
        _lib().rt.memcpy_h2d(out.data_ptr(), a.ctypes.data, a.nbytes, N.stream(dev.index))
    return out


# --------------------------------------------------------------------- copies
def copy_(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """dst[...] = src (broadcast to dst's shape, converted to dst's dtype),
    any strides on either side."""
    if dst.numel() == 0:
        return dst
    if not on_gpu(dst, src):
        if CP.copy_ok(dst, src) and not src.is_cuda and not dst.is_cuda and src.dtype != torch.bool:
            if src.data_ptr() == dst.data_ptr() and src.dtype == dst.dtype and src.stride() == dst.stride() \
                    and src.shape == dst.shape:
                return dst
            shape = tuple(dst.shape)
            size, ds, ss = coalesce(shape, list(dst.stride()), _bstrides(src, shape))
            CP.lib().copy_nd(src.data_ptr(), CP.dt(src), dst.data_ptr(), CP.dt(dst), size, ds, ss)
            return dst
        return dst.copy_(src)
    if not (src.is_cuda and dst.is_cuda):
        if src.is_cuda == dst.is_cuda:
            return dst.copy_(src)
        # host <-> device: the DMA engine (memcpy), then a native layout pass if needed
        staged = src.to(dst.device) if not src.is_cuda else src.cpu()
        return copy_(dst, staged) if staged.is_cuda else dst.copy_(staged)
    shape = tuple(dst.shape)
    size, ds, ss = coalesce(shape, list(dst.stride()), _bstrides(src, shape))
    _lib().copy_nd(src.data_ptr(), N.dt(src), dst.data_ptr(), N.dt(dst), size, ds, ss, N.stream())
    return dst


def empty_like_fmt(t: torch.Tensor, dtype=None, memory_format=torch.contiguous_format) -> torch.Tensor:
    return _mem.empty(t.shape, dtype=dtype or t.dtype, device=t.device, memory_format=memory_format)


def contiguous(t: torch.Tensor, memory_format=torch.contiguous_format) -> torch.Tensor:
    """Dense copy in the requested memory format (no-op if already dense)."""
    if t.is_contiguous(memory_format=memory_format):
        return t
    if not on_gpu(t) and not CP.copy_ok(t):
        return t.contiguous(memory_format=memory_format)
    return copy_(empty_like_fmt(t, memory_format=memory_format), t)


def dense(t: torch.Tensor) -> torch.Tensor:
    """Dense in either row-major or channels-last order (whichever it is closest to)."""
    if t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)):
        return t
    return contiguous(t)


def to(t: torch.Tensor, dtype: Optional[torch.dtype] = None, memory_format=None) -> torch.Tensor:
    """dtype / memory-format conversion in one pass."""
    dtype = dtype or t.dtype
    if memory_format is None:
        if t.dtype == dtype:
            return t
        fmt = torch.channels_last if (t.dim() == 4 and not t.is_contiguous()
                                      and t.is_contiguous(memory_format=torch.channels_last)) else torch.contiguous_format
    else:
        fmt = memory_format
        if t.dtype == dtype and t.is_contiguous(memory_format=fmt):
            return t
    if not on_gpu(t) and not (CP.copy_ok(t) and dtype in CP._DT and t.dtype != torch.bool):
        return t.to(dtype=dtype, memory_format=fmt)
    return copy_(_mem.empty(t.shape, dtype=dtype, device=t.device, memory_format=fmt), t)


def reshape(t: torch.Tensor, shape) -> torch.Tensor:
    """A view when the strides allow it, else one native dense copy first."""
    try:
        return t.view(shape)
    except RuntimeError:
        return contiguous(t).view(shape)


# --------------------------------------------------------------------- fills
def fill_(t: torch.Tensor, value: float) -> torch.Tensor:
    if CP.copy_ok(t) and t.is_contiguous():
        if t.numel():
            CP.lib().fill(t.data_ptr(), t.numel(), CP.dt(t), float(value))
        return t
    if not on_gpu(t) or not t.is_contiguous() and not (t.dim() == 4 and
                                                       t.is_contiguous(memory_format=torch.channels_last)):
        if on_gpu(t) or CP.copy_ok(t):
            return copy_(t, full((), value, t.dtype, t.device))  # broadcast (stride-0) copy into the strided view
        return t.fill_(value)
    if t.numel():
        _lib().fill(t.data_ptr(), t.numel(), N.dt(t), float(value), N.stream())
    return t


def zero_(t: torch.Tensor) -> torch.Tensor:
    return fill_(t, 0.0)


def iadd_(t: torch.Tensor, v: int) -> torch.Tensor:
    """In-place integer increment of a dense int64 device counter."""
    if on_gpu(t) and t.dtype == torch.int64 and t.is_contiguous():
        _lib().iadd_i64(t.data_ptr(), t.numel(), int(v), N.stream())
        return t
    return t.add_(v)


def random_(t: torch.Tensor, dist: str, a: float, b: float, device_obj=None) -> torch.Tensor:
    """Fill t with uniform [a, b) or gaussian (mean a, std b) samples: the
    Philox kernel on the GPU (counters reserved from the SINGA device's
    stream, reproducible per seed), the device's torch generator on the CPU."""
    if on_gpu(t) and t.dtype in _FLOATS:
        seed, off = device_obj.next_rng(t.numel()) if device_obj is not None else (0, 0)
        d = t if t.is_contiguous() else _mem.empty(t.shape, dtype=t.dtype, device=t.device)
        if d.numel():
            _lib().rand_fill(d.data_ptr(), d.numel(), N.dt(d), 0 if dist == "uniform" else 1, float(a), float(b),
                             int(seed), int(off), N.stream())
        return t if d is t else copy_(t, d)
    if not t.is_cuda and CP.lib() is not None and t.dtype == torch.float32:
        # the same Philox stream as the GPU kernel (in oracle mode too: the
        # initial weights of a native run and its oracle run are identical)
        seed, off = device_obj.next_rng(t.numel()) if device_obj is not None else (0, 0)
        d = t if t.is_contiguous() else _mem.empty(t.shape, dtype=torch.float32)
        if d.numel():
            CP.lib().rand_fill(d.data_ptr(), d.numel(), 0 if dist == "uniform" else 1, float(a), float(b), int(seed),
                               int(off))
        return t if d is t else copy_(t, d)
    gen = device_obj.generator if device_obj is not None else None
    d = _mem.empty(t.shape, dtype=torch.float32, device=t.device)
    if dist == "uniform":
        d.uniform_(a, b, generator=gen)
    else:
        d.normal_(a, b, generator=gen)
    return t.copy_(d)


def full(shape, value, dtype, device, memory_format=torch.contiguous_format) -> torch.Tensor:
    t = _mem.empty(tuple(shape), dtype=dtype, device=device, memory_format=memory_format)
    if t.is_cuda and N.force_native():
        if t.numel():
            _lib().fill(t.data_ptr(), t.numel(), N.dt(t), float(value), N.stream())
        return t
    if CP.copy_ok(t):
        if t.numel():
            CP.lib().fill(t.data_ptr(), t.numel(), CP.dt(t), float(value))
        return t
    return t.fill_(value)


def zeros(shape, dtype=torch.float32, device="cpu", memory_format=torch.contiguous_format) -> torch.Tensor:
    return full(shape, 0.0, dtype, device, memory_format)


def zeros_like(t: torch.Tensor, dtype=None) -> torch.Tensor:
    fmt = torch.channels_last if (t.dim() == 4 and not t.is_contiguous()
                                  and t.is_contiguous(memory_format=torch.channels_last)) else torch.contiguous_format
    return zeros(t.shape, dtype or t.dtype, t.device, fmt)


# --------------------------------------------------------------------- elementwise
def binary(op: str, a: torch.Tensor, b, out_dtype: Optional[torch.dtype] = None, alpha: float = 1.0,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """alpha * (a OP b) with NumPy broadcasting; comparisons / logic give 0/1
    in the float dtype.  b may be a Python scalar."""
    if not isinstance(b, torch.Tensor):  # a scalar: a fill kernel on the GPU (graph-capturable, no H2D copy)
        b = full((), float(b), a.dtype if a.is_floating_point() else torch.float32, a.device)
    dt = a.dtype if a.dtype == b.dtype else (torch.float32 if torch.float32 in (a.dtype, b.dtype) else a.dtype)
    if on_gpu(a, b) and dt in _FLOATS and a.is_cuda and b.is_cuda:
        a = to(a, dt) if a.dtype != dt else a
        b = to(b, dt) if b.dtype != dt else b
        shape = tuple(torch.broadcast_shapes(a.shape, b.shape))
        if out is None:
            out = _mem.empty(shape, dtype=dt, device=a.device)
        size, os_, as_, bs_ = coalesce(shape, list(out.stride()), _bstrides(a, shape), _bstrides(b, shape))
        _lib().binary_nd(BIN[op], a.data_ptr(), b.data_ptr(), out.data_ptr(), N.dt(out), size, os_, as_, bs_,
                         float(alpha), N.stream())
        if out_dtype is not None and out_dtype != out.dtype:
            return to(out, out_dtype)
        return out
    if on_gpu(a, b):
        raise NotImplementedError(f"binary {op}: no native kernel for {a.dtype} x {b.dtype}")
    od = out_dtype or dt
    if CP.ok(out) and CP.copy_ok(a, b) and (out is not None or od == torch.float32) and a.dtype != torch.bool \
            and b.dtype != torch.bool:
        a = a if a.dtype == torch.float32 else to(a, torch.float32)
        b = b if b.dtype == torch.float32 else to(b, torch.float32)
        shape = tuple(torch.broadcast_shapes(a.shape, b.shape))
        o = out if out is not None and tuple(out.shape) == shape else _mem.empty(shape, dtype=torch.float32)
        size, os_, as_, bs_ = coalesce(shape, list(o.stride()), _bstrides(a, shape), _bstrides(b, shape))
        CP.lib().binary_nd(BIN[op], a.data_ptr(), b.data_ptr(), o.data_ptr(), size, os_, as_, bs_, float(alpha))
        if out is not None and o is not out:
            return copy_(out, o)
        return o
    af, bf = a.float(), b.float()
    r = {"add": lambda: af + bf, "sub": lambda: af - bf, "mul": lambda: af * bf, "div": lambda: af / bf,
         "pow": lambda: torch.pow(af, bf), "max": lambda: torch.maximum(af, bf), "min": lambda: torch.minimum(af, bf),
         "lt": lambda: (af < bf).float(), "le": lambda: (af <= bf).float(), "gt": lambda: (af > bf).float(),
         "ge": lambda: (af >= bf).float(), "eq": lambda: (af == bf).float(), "ne": lambda: (af != bf).float(),
         "and": lambda: ((af != 0) & (bf != 0)).float(), "or": lambda: ((af != 0) | (bf != 0)).float(),
         "xor": lambda: ((af != 0) ^ (bf != 0)).float()}[op]()
    if alpha != 1.0:
        r = r * alpha
    r = r.to(out_dtype or dt)
    if out is not None:
        return out.copy_(r)
    return r


def where(cond: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """cond ? a : b with broadcasting (cond: any dtype, non-zero = true)."""
    dt = a.dtype if a.dtype == b.dtype else torch.float32
    if on_gpu(cond, a, b) and (dt in _FLOATS or dt == torch.int64):
        c = cond if cond.dtype in (torch.uint8, torch.bool) else binary("ne", to(cond, torch.float32), 0.0)
        if c.dtype not in (torch.uint8, torch.bool):
            c = to(c, torch.uint8)
        if c.dtype == torch.bool:
            c = c.view(torch.uint8)
        a, b = to(a, dt), to(b, dt)
        shape = tuple(torch.broadcast_shapes(c.shape, a.shape, b.shape))
        out = _mem.empty(shape, dtype=dt, device=a.device)
        size, os_, as_, bs_, cs_ = coalesce(shape, list(out.stride()), _bstrides(a, shape), _bstrides(b, shape),
                                            _bstrides(c, shape))
        _lib().where_nd(c.data_ptr(), a.data_ptr(), b.data_ptr(), out.data_ptr(), N.dt(out), size, os_, as_, bs_,
                        cs_, N.stream())
        return out
    if on_gpu(cond, a, b):
        raise NotImplementedError(f"where: no native kernel for {dt}")
    if CP.copy_ok(cond, a, b) and dt == torch.float32:
        c = cond if cond.dtype in (torch.uint8, torch.bool) else binary("ne", to(cond, torch.float32), 0.0)
        if c.dtype == torch.bool:
            c = c.view(torch.uint8)
        elif c.dtype != torch.uint8:
            c = to(c, torch.uint8)
        a, b = to(a, dt), to(b, dt)
        shape = tuple(torch.broadcast_shapes(c.shape, a.shape, b.shape))
        out = _mem.empty(shape, dtype=dt)
        size, os_, as_, bs_, cs_ = coalesce(shape, list(out.stride()), _bstrides(a, shape), _bstrides(b, shape),
                                            _bstrides(c, shape))
        CP.lib().where_nd(c.data_ptr(), a.data_ptr(), b.data_ptr(), out.data_ptr(), size, os_, as_, bs_, cs_)
        return out
    return torch.where(cond.bool(), a.to(dt), b.to(dt))


def unary(op: str, x: torch.Tensor, alpha: float = 0.0) -> torch.Tensor:
    from . import functional as F
    return F.unary(op, x, alpha)


def clamp_affine(x: torch.Tensor, a: float = 1.0, b: float = 0.0, lo: float = -math.inf, hi: float = math.inf,
                 dy: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = clamp(a x + b, lo, hi) (clip, hardsigmoid, relu6); with dy: its
    gradient dy * a inside the open interval."""
    if on_gpu(x) and x.dtype in _FLOATS:
        x = dense(x)
        g = None
        if dy is not None:
            g = dy if (dy.dtype == x.dtype and dy.stride() == x.stride()) else copy_(_mem.empty_like(x), dy)
        out = _mem.empty_like(x)
        _lib().clamp_affine(x.data_ptr(), N.ptr(g), out.data_ptr(), x.numel(), N.dt(x), float(a), float(b),
                            float(max(lo, -3.4e38)), float(min(hi, 3.4e38)), N.stream())
        return out
    if on_gpu(x):
        raise NotImplementedError(f"clamp_affine: no native kernel for {x.dtype}")
    if CP.ok(x, dy):
        xc = CP.dense32(x)
        g = CP.dense32(dy) if dy is not None else None
        out = _mem.empty(x.shape, dtype=torch.float32)
        CP.lib().clamp_affine(xc.data_ptr(), CP.p(g), out.data_ptr(), xc.numel(), float(a), float(b),
                              float(max(lo, -3.4e38)), float(min(hi, 3.4e38)))
        return out
    z = a * x.float() + b
    if dy is None:
        return torch.clamp(z, lo, hi).to(x.dtype)
    return (dy.float() * a * ((z > lo) & (z < hi)).float()).to(x.dtype)


# --------------------------------------------------------------------- reductions
def reduce(x: torch.Tensor, axes: Optional[Sequence[int]] = None, op: str = "sum", keepdims: bool = False,
           out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """sum / mean / max / min / sumsq over `axes` (None: all).  The reduced
    axes are made adjacent (one native permute copy if they are not), then
    one [outer][red][inner] reduction."""
    nd = x.dim()
    axes = list(range(nd)) if axes is None else sorted({a % nd for a in axes}) if nd else []
    od = out_dtype or (x.dtype if x.dtype in _FLOATS else torch.float32)
    oshape = [1 if k in axes else s for k, s in enumerate(x.shape)] if keepdims else \
        [s for k, s in enumerate(x.shape) if k not in axes]
    if not axes:
        return to(x, od).clone() if x.dtype == od else to(x, od)
    host = CP.copy_ok(x) and x.dtype != torch.bool and od in _FLOATS
    if (on_gpu(x) and x.dtype in _FLOATS and od in _FLOATS) or host:
        if host and x.dtype != torch.float32:
            x = to(x, torch.float32)
        keep = [k for k in range(nd) if k not in axes]
        lo, hi = min(axes), max(axes)
        if axes == list(range(lo, hi + 1)):  # already adjacent
            xc = contiguous(x)
            outer = int(math.prod(x.shape[:lo]))
            red = int(math.prod(x.shape[lo:hi + 1]))
            inner = int(math.prod(x.shape[hi + 1:]))
        else:  # kept dims first, reduced dims last
            xc = contiguous(x.permute(*keep, *axes))
            outer = int(math.prod(x.shape[k] for k in keep))
            red = int(math.prod(x.shape[k] for k in axes))
            inner = 1
        y = _mem.empty(oshape, dtype=od, device=x.device)
        if y.numel() == 0:
            return y
        if red == 0:
            return fill_(y, 0.0 if op in ("sum", "mean", "sumsq") else float("nan"))
        if host:
            y32 = y if y.dtype == torch.float32 else _mem.empty(oshape, dtype=torch.float32)
            CP.lib().reduce(xc.data_ptr(), y32.data_ptr(), outer, red, inner, RED[op])
            return y if y32 is y else copy_(y, y32)
        _lib().reduce(xc.data_ptr(), N.dt(xc), y.data_ptr(), N.dt(y), outer, red, inner, RED[op], N.stream())
        return y
    if on_gpu(x):
        raise NotImplementedError(f"reduce {op}: no native kernel for {x.dtype}")
    xf = x.float()
    r = {"sum": lambda: xf.sum(dim=axes, keepdim=keepdims), "mean": lambda: xf.mean(dim=axes, keepdim=keepdims),
         "sumsq": lambda: (xf * xf).sum(dim=axes, keepdim=keepdims),
         "max": lambda: xf.amax(dim=axes, keepdim=keepdims), "min": lambda: xf.amin(dim=axes, keepdim=keepdims)}[op]()
    return r.to(od).reshape(oshape)


def sum_to(g: torch.Tensor, shape) -> torch.Tensor:
    """Reduce a broadcast result's gradient back to `shape` (NumPy rules)."""
    shape = tuple(shape)
    if tuple(g.shape) == shape:
        return g
    lead = g.dim() - len(shape)
    axes = list(range(lead)) + [lead + k for k, s in enumerate(shape) if s == 1 and g.shape[lead + k] != 1]
    r = reduce(g, axes, "sum", keepdims=True, out_dtype=g.dtype if g.dtype in _FLOATS else torch.float32)
    return r.reshape(shape)


# --------------------------------------------------------------------- concat / slices / tiles
def cat(ts: Sequence[torch.Tensor], axis: int = 0) -> torch.Tensor:
    ts = list(ts)
    if not on_gpu(*ts) and not CP.copy_ok(*ts):
        return torch.cat(ts, dim=axis)  # (a host dtype without a native conversion, or the test oracle)
    nd = ts[0].dim()
    axis %= nd
    # mixed dtypes: PyTorch's promotion, every part converted by the native copy
    dt = ts[0].dtype if len({t.dtype for t in ts}) == 1 else _promote([t.dtype for t in ts])
    shape = list(ts[0].shape)
    shape[axis] = sum(t.shape[axis] for t in ts)
    out = _mem.empty(shape, dtype=dt, device=ts[0].device)
    o = 0
    for t in ts:
        n = t.shape[axis]
        if n:
            copy_(out.narrow(axis, o, n), t)
        o += n
    return out


def scatter_slices(parts: Sequence[Optional[torch.Tensor]], sizes: Sequence[int], axis: int, like: torch.Tensor):
    """The gradient of a split: the parts concatenated, zeros where a part
    has no gradient."""
    if all(p is not None for p in parts):
        return cat(parts, axis)
    shape = list(like.shape)
    out = zeros(shape, like.dtype, like.device)
    o = 0
    for p, n in zip(parts, sizes):
        if p is not None and n:
            copy_(out.narrow(axis, o, n), p)
        o += n
    return out


def tile(x: torch.Tensor, repeats: Sequence[int]) -> torch.Tensor:
    """np.tile / torch.repeat: out viewed as [r0, s0, r1, s1, ...] with the
    source broadcast (stride 0) over the r dims -- one copy."""
    reps = list(repeats)
    if len(reps) < x.dim():
        reps = [1] * (x.dim() - len(reps)) + reps
    xs = reshape(x, (1,) * (len(reps) - x.dim()) + tuple(x.shape))
    if not on_gpu(x) and not CP.copy_ok(x):
        return xs.repeat(*reps)
    inter = []
    for r, s in zip(reps, xs.shape):
        inter += [r, s]
    out = _mem.empty(inter, dtype=x.dtype, device=x.device)
    src = xs.reshape([v for s in xs.shape for v in (1, s)]).expand(*inter)
    copy_(out, src)
    return out.reshape([r * s for r, s in zip(reps, xs.shape)])


def tile_backward(g: torch.Tensor, repeats: Sequence[int], in_shape) -> torch.Tensor:
    reps = list(repeats)
    nd = max(len(reps), len(in_shape))
    reps = [1] * (nd - len(reps)) + reps
    base = (1,) * (nd - len(in_shape)) + tuple(in_shape)
    inter = []
    for r, s in zip(reps, base):
        inter += [r, s]
    gg = reshape(g, inter)
    r = reduce(gg, [2 * k for k in range(nd)], "sum", keepdims=False, out_dtype=g.dtype)
    return r.reshape(in_shape)


def expand(x: torch.Tensor, shape) -> torch.Tensor:
    """Dense broadcast of x to `shape`."""
    shape = tuple(shape)
    if tuple(x.shape) == shape:
        return x
    if not on_gpu(x) and not CP.copy_ok(x):
        return x.expand(*shape).contiguous()
    out = _mem.empty(shape, dtype=x.dtype, device=x.device)
    return copy_(out, x.expand(*shape) if x.dim() == len(shape) else x)


# --------------------------------------------------------------------- gathers / scatters
def _idx(idx: torch.Tensor, device) -> torch.Tensor:
    if idx.device != device:
        idx = idx.to(device)
    if idx.dtype not in (torch.int32, torch.int64):
        idx = idx.long()
    return contiguous(idx)


def _promote(dts):
    out = dts[0]
    for d in dts[1:]:
        out = torch.promote_types(out, d)
    return out


def index_select(x: torch.Tensor, axis: int, idx: torch.Tensor) -> torch.Tensor:
    """out = x.take(idx, axis) with out.shape = x.shape[:axis] + idx.shape + x.shape[axis+1:]."""
    axis %= x.dim()
    if not on_gpu(x) and CP.copy_ok(x) and not idx.is_cuda and idx.dtype not in (torch.int32, torch.int64):
        import numpy as np  # other host index dtypes: converted on the host (no torch kernel)
        idx = torch.from_numpy(np.ascontiguousarray(idx.numpy(), np.int64))
    if not on_gpu(x) and CP.copy_ok(x) and idx.is_cuda and idx.dtype in (torch.int32, torch.int64):
        idx = idx.cpu()  # (indices of a host gather: one small device -> host copy)
    if not on_gpu(x) and CP.copy_ok(x) and not idx.is_cuda and idx.dtype in (torch.int32, torch.int64):
        xc, ic = contiguous(x), contiguous(idx)
        outer = int(math.prod(x.shape[:axis]))
        inner = int(math.prod(x.shape[axis + 1:]))
        out = _mem.empty(x.shape[:axis] + tuple(idx.shape) + x.shape[axis + 1:], dtype=x.dtype)
        if out.numel():
            CP.lib().index_select(xc.data_ptr(), ic.data_ptr(), int(ic.dtype == torch.int64), out.data_ptr(), outer,
                                  x.shape[axis], inner, ic.numel(), x.element_size())
        return out
    if not on_gpu(x):
        r = torch.index_select(x, axis, idx.reshape(-1).long().to(x.device))
        return r.reshape(x.shape[:axis] + tuple(idx.shape) + x.shape[axis + 1:])
    idx = _idx(idx, x.device)
    xc = contiguous(x)
    outer = int(math.prod(x.shape[:axis]))
    inner = int(math.prod(x.shape[axis + 1:]))
    out = _mem.empty(x.shape[:axis] + tuple(idx.shape) + x.shape[axis + 1:], dtype=x.dtype, device=x.device)
    if out.numel():
        _lib().index_select(xc.data_ptr(), idx.data_ptr(), int(idx.dtype == torch.int64), out.data_ptr(), outer,
                            x.shape[axis], inner, idx.numel(), x.element_size(), N.stream())
    return out


def index_add_(dst: torch.Tensor, axis: int, idx: torch.Tensor, src: torch.Tensor, alpha: float = 1.0) -> torch.Tensor:
    """dst.index_add_(axis, idx, src) into an fp32 dense dst (atomics)."""
    axis %= dst.dim()
    if (not on_gpu(dst) and CP.ok(dst) and dst.is_contiguous() and CP.copy_ok(src) and not idx.is_cuda
            and idx.dtype in (torch.int32, torch.int64)):
        s = src if src.dtype == torch.float32 and src.is_contiguous() else to(contiguous(src), torch.float32)
        ic = contiguous(idx)
        outer = int(math.prod(dst.shape[:axis]))
        inner = int(math.prod(dst.shape[axis + 1:]))
        if s.numel():
            CP.lib().index_add(dst.data_ptr(), ic.data_ptr(), int(ic.dtype == torch.int64), s.data_ptr(), outer,
                               dst.shape[axis], inner, ic.numel(), float(alpha))
        return dst
    if not on_gpu(dst):
        s = src.reshape(dst.shape[:axis] + (idx.numel(),) + dst.shape[axis + 1:]).to(dst.dtype)
        return dst.index_add_(axis, idx.reshape(-1).long(), s, alpha=alpha)
    if dst.dtype != torch.float32 or not dst.is_contiguous():
        raise ValueError("index_add_: native path needs a dense fp32 destination")
    idx = _idx(idx, dst.device)
    s = contiguous(src)
    if s.dtype not in _FLOATS:
        s = to(s, torch.float32)
    outer = int(math.prod(dst.shape[:axis]))
    inner = int(math.prod(dst.shape[axis + 1:]))
    if s.numel():
        _lib().index_add(dst.data_ptr(), idx.data_ptr(), int(idx.dtype == torch.int64), s.data_ptr(), N.dt(s), outer,
                         dst.shape[axis], inner, idx.numel(), float(alpha), N.stream())
    return dst


def gather_elements(x: torch.Tensor, axis: int, idx: torch.Tensor) -> torch.Tensor:
    axis %= x.dim()
    if not on_gpu(x):
        return torch.gather(x, axis, idx.long())
    xc, ic = contiguous(x), _idx(idx, x.device)
    outer = int(math.prod(idx.shape[:axis]))
    inner = int(math.prod(idx.shape[axis + 1:]))
    if tuple(x.shape[:axis]) != tuple(idx.shape[:axis]) or tuple(x.shape[axis + 1:]) != tuple(idx.shape[axis + 1:]):
        raise NotImplementedError("gather_elements: index shape must match the data outside the axis")
    out = _mem.empty(idx.shape, dtype=x.dtype, device=x.device)
    _lib().gather_el(xc.data_ptr(), ic.data_ptr(), int(ic.dtype == torch.int64), out.data_ptr(), N.dt(x), outer,
                     x.shape[axis], idx.shape[axis], inner, N.stream())
    return out


def scatter_elements(x: torch.Tensor, axis: int, idx: torch.Tensor, upd: torch.Tensor, add: bool = False):
    """out = x with out[.. idx ..] = upd (or += with add, fp32) along axis."""
    axis %= x.dim()
    if not on_gpu(x):
        return x.scatter_add(axis, idx.long(), upd) if add else x.scatter(axis, idx.long(), upd)
    out = contiguous(x).clone() if x.is_contiguous() else contiguous(x)
    ic, uc = _idx(idx, x.device), contiguous(to(upd, x.dtype))
    if tuple(x.shape[:axis]) != tuple(idx.shape[:axis]) or tuple(x.shape[axis + 1:]) != tuple(idx.shape[axis + 1:]):
        raise NotImplementedError("scatter_elements: index shape must match the data outside the axis")
    outer = int(math.prod(idx.shape[:axis]))
    inner = int(math.prod(idx.shape[axis + 1:]))
    _lib().scatter_el(out.data_ptr(), ic.data_ptr(), int(ic.dtype == torch.int64), uc.data_ptr(), N.dt(out), outer,
                      x.shape[axis], idx.shape[axis], inner, int(add), N.stream())
    return out


# --------------------------------------------------------------------- padding
def _pad_maps(isz, osz, before, mode):
    """Per-dim output -> input index maps of reflect / edge padding (CPU reference)."""
    import numpy as np
    maps = []
    for n, o, b in zip(isz, osz, before):
        i = np.arange(o) - b
        if mode == "edge":
            i = np.clip(i, 0, n - 1)
        elif n == 1:
            i = np.zeros_like(i)
        else:
            p = 2 * (n - 1)
            m = np.mod(i, p)
            i = np.where(m < n, m, p - m)
        maps.append(i)
    return maps


def pad(x: torch.Tensor, before: Sequence[int], after: Sequence[int], mode: str = "constant",
        value: float = 0.0) -> torch.Tensor:
    """N-d pad (ONNX Pad semantics: per-dim before / after counts, modes
    constant / reflect / edge)."""
    nd = x.dim()
    osz = [s + b + a for s, b, a in zip(x.shape, before, after)]
    if not on_gpu(x) and mode == "constant" and CP.copy_ok(x) and min(list(before) + list(after) + [0]) >= 0:
        y = full(osz, value, x.dtype, x.device)
        v = y
        for k in range(nd):
            v = v.narrow(k, before[k], x.shape[k])
        copy_(v, x)
        return y
    if not on_gpu(x) and CP.copy_ok(x) and mode == "constant":
        # negative counts crop: narrow first, then the native constant pad
        v = x
        for k in range(nd):
            b0, a0 = min(before[k], 0), min(after[k], 0)
            if b0 or a0:
                v = v.narrow(k, -b0, v.shape[k] + b0 + a0)
        return pad(contiguous(v), [max(b, 0) for b in before], [max(a, 0) for a in after], mode, value)
    if not on_gpu(x) and CP.copy_ok(x):
        # reflect / edge: one native gather per padded dim through the index maps
        import numpy as np
        maps = _pad_maps(x.shape, osz, before, mode)
        y = x
        for k, m in enumerate(maps):
            if len(m) != x.shape[k] or np.any(m != np.arange(x.shape[k])):
                y = index_select(y, k, torch.from_numpy(np.ascontiguousarray(m, np.int64)))
        return y
    if not on_gpu(x):
        if mode == "constant":
            tp = []
            for i in reversed(range(nd)):
                tp += [before[i], after[i]]
            return torch.nn.functional.pad(x, tp, mode="constant", value=value)
        maps = _pad_maps(x.shape, osz, before, mode)
        return x[torch.meshgrid(*[torch.as_tensor(m) for m in maps], indexing="ij")]
    y = _mem.empty(osz, dtype=x.dtype, device=x.device)
    _lib().pad_nd(x.data_ptr(), y.data_ptr(), N.dt(x), osz, list(x.shape), list(x.stride()), list(before), PAD[mode],
                  float(value), N.stream())
    return y


def pad_backward(dy: torch.Tensor, in_shape, before: Sequence[int], mode: str = "constant") -> torch.Tensor:
    nd = len(in_shape)
    if mode == "constant":  # the interior slice
        v = dy
        for k in range(nd):
            v = v.narrow(k, before[k], in_shape[k])
        return contiguous(v)
    if not on_gpu(dy):
        maps = _pad_maps(in_shape, dy.shape, before, mode)
        dx = torch.zeros(in_shape, dtype=torch.float32)
        dx.index_put_(torch.meshgrid(*[torch.as_tensor(m) for m in maps], indexing="ij"), dy.float(), accumulate=True)
        return dx.to(dy.dtype)
    dyc = contiguous(dy)
    dx = zeros(in_shape, torch.float32, dy.device)
    _lib().pad_bwd(dyc.data_ptr(), dx.data_ptr(), N.dt(dyc), list(dy.shape), list(in_shape), list(dx.stride()),
                   list(before), PAD[mode], N.stream())
    return dx if dy.dtype == torch.float32 else to(dx, dy.dtype)


# --------------------------------------------------------------------- selection
_KTH_WS: dict = {}


def kth_largest_abs(x: torch.Tensor, k: int) -> torch.Tensor:
    """0-d fp32 tensor holding the k-th largest |x| (exact): a 3-pass radix
    select on the device (no sort, no host sync), graph-capturable."""
    if not on_gpu(x):
        a = x.float().abs().reshape(-1)
        return a.kthvalue(a.numel() - int(k) + 1).values
    if x.dtype != torch.float32:
        x = to(x, torch.float32)
    x = contiguous(x)
    key = (x.device, torch.cuda.current_stream(x.device).cuda_stream)
    ws = _KTH_WS.get(key)
    if ws is None:
        ws = _KTH_WS[key] = _mem.empty(2048 + 2, dtype=torch.int32, device=x.device)
    out = _mem.empty((), dtype=torch.float32, device=x.device)
    _lib().kth_largest_abs(x.data_ptr(), x.numel(), int(k), out.data_ptr(), ws.data_ptr(), N.stream())
    return out
