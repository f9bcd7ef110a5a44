"""Device-dispatching functional ops on raw ``torch.Tensor`` storage.

Every op has two implementations:

* GPU (``tensor.is_cuda``): a hand-written gfx950 HIP kernel from
  ``singa_amd/csrc/kernels`` launched on the current HIP stream.  Activation
  tensors of 4-D ops are NHWC in memory (``torch.channels_last``) while the
  logical shape stays NCHW as in SINGA's API.  bf16 convolutions / GEMMs of
  aligned shapes run the tuned MFMA kernels (igemm.hip); fp32 operands run
  the exact-f32 MFMA kernels (ggemm.hip) -- no silent downcast -- as do
  ragged bf16 shapes, grouped and dilated convolutions.  A GPU case without a
  native kernel RAISES (``_no_native``); nothing falls back to PyTorch /
  hipBLAS / MIOpen on the device.
* CPU (the ``CppCPU`` device): fp32 host tensors run the native C++
  kernels of ``_core.cpu`` (csrc/runtime/cpu_ops.cc, dispatched by
  :mod:`singa_amd.ops.cpu`).  The plain PyTorch expressions below each native
  branch are the numerics ORACLE of the tests (``cpu.torch_oracle()``) and
  the path of host dtypes without a native kernel (bf16 on the CPU).
"""
from __future__ import annotations

import math
import os
import threading
from typing import Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from .. import memory as _mem
from . import cpu as CP
from . import glue as G
from . import native as N

# unary op codes (csrc/kernels/elementwise.hip)
UNARY = {"relu": 0, "sigmoid": 1, "tanh": 2, "stanh": 3, "gelu": 4, "identity": 5, "softplus": 6, "square": 7,
         "abs": 8, "exp": 9, "leakyrelu": 10, "elu": 11, "selu": 12, "gelu_tanh": 13, "sqrt": 14, "neg": 15,
         "reciprocal": 16, "log": 17, "sign": 18, "erf": 19, "cos": 20, "sin": 21, "tan": 22, "cosh": 23,
         "sinh": 24, "acos": 25, "asin": 26, "atan": 27, "acosh": 28, "asinh": 29, "atanh": 30, "ceil": 31,
         "floor": 32, "round": 33, "softsign": 34, "scale": 35, "adds": 36, "rsqrt": 37, "pows": 38}

_CPU_UNARY = {
    "relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh,
    "stanh": lambda x: 1.7159047 * torch.tanh(0.66666667 * x),
    "gelu": lambda x: F.gelu(x), "gelu_tanh": lambda x: F.gelu(x, approximate="tanh"),
    "identity": lambda x: x.clone(), "softplus": F.softplus, "square": torch.square, "abs": torch.abs,
    "exp": torch.exp, "sqrt": torch.sqrt, "neg": torch.neg, "reciprocal": torch.reciprocal, "log": torch.log,
    "sign": torch.sign, "erf": torch.erf, "cos": torch.cos, "sin": torch.sin, "tan": torch.tan, "cosh": torch.cosh,
    "sinh": torch.sinh, "acos": torch.acos, "asin": torch.asin, "atan": torch.atan, "acosh": torch.acosh,
    "asinh": torch.asinh, "atanh": torch.atanh, "ceil": torch.ceil, "floor": torch.floor, "round": torch.round,
    "softsign": lambda x: x / (1 + x.abs()), "rsqrt": torch.rsqrt,
}


def _native_ok(*ts: torch.Tensor) -> bool:
    return all(t is None or t.is_cuda for t in ts) and N.force_native()


def _flat_ok(t: torch.Tensor) -> bool:
    return t.dtype in (torch.float32, torch.bfloat16) and (t.is_contiguous() or N.is_cl(t))


_NO_BN_STATS = os.environ.get("SG_NO_BN_STATS", "0") == "1"


def _same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same shape and the same dense element order (strides of size-1 dims
    do not matter: [N,C,1,1] is both NCHW- and NHWC-dense)."""
    if a.shape != b.shape:
        return False
    if a.stride() == b.stride():
        return True
    if a.is_contiguous() and b.is_contiguous():
        return True
    return a.dim() == 4 and N.is_cl(a) and N.is_cl(b)


def _like(t: torch.Tensor, dtype=None) -> torch.Tensor:
    """Empty tensor with the same shape AND memory layout as t."""
    if t.dim() == 4 and N.is_cl(t) and not t.is_contiguous():
        return _mem.empty(t.shape, dtype=dtype or t.dtype, device=t.device, memory_format=torch.channels_last)
    return _mem.empty(t.shape, dtype=dtype or t.dtype, device=t.device)


def _zeros_cl(shape, dtype, device) -> torch.Tensor:
    return G.zeros(shape, dtype, device, torch.channels_last)


def _dense(t: torch.Tensor) -> torch.Tensor:
    return G.dense(t)


# ----------------------------------------------------------------------------
# elementwise
# ----------------------------------------------------------------------------
def unary(op: str, x: torch.Tensor, alpha: float = 0.0) -> torch.Tensor:
    if _native_ok(x) and x.dtype in (torch.float32, torch.bfloat16) and op in UNARY:
        x = G.dense(x)
        y = _like(x)
        N.lib().unary_fwd(UNARY[op], x.data_ptr(), y.data_ptr(), x.numel(), N.dt(x), alpha, N.stream())
        return y
    _no_native(f"unary {op}", x)
    if CP.ok(x) and op in UNARY:
        x = CP.dense32(x)
        y = _mem.empty(x.shape, dtype=torch.float32)
        CP.lib().unary_fwd(UNARY[op], x.data_ptr(), y.data_ptr(), x.numel(), float(alpha))
        return y
    if op == "leakyrelu":
        return F.leaky_relu(x, alpha)
    if op == "elu":
        return F.elu(x, alpha)
    if op == "selu":
        return F.selu(x)
    if op == "scale":
        return x * alpha
    if op == "adds":
        return x + alpha
    if op == "pows":
        return torch.pow(x, alpha)
    return _CPU_UNARY[op](x)


def unary_bwd(op: str, x: Optional[torch.Tensor], y: Optional[torch.Tensor], dy: torch.Tensor,
              alpha: float = 0.0) -> torch.Tensor:
    if _native_ok(dy) and dy.dtype in (torch.float32, torch.bfloat16) and op in UNARY:
        dy = G.dense(dy)
        xx = G.dense(x) if x is not None else None
        yy = G.dense(y) if y is not None else None
        for t in (xx, yy):
            if t is not None and not _same_layout(t, dy):
                raise ValueError("unary_bwd: layout mismatch")
        dx = _like(dy)
        N.lib().unary_bwd(UNARY[op], N.ptr(xx), N.ptr(yy), dy.data_ptr(), dx.data_ptr(), dy.numel(), N.dt(dy),
                          alpha, N.stream())
        return dx
    _no_native(f"unary_bwd {op}", dy)
    if CP.ok(x, y, dy) and op in UNARY:
        dy = CP.dense32(dy)
        xx = CP.dense32(x) if x is not None else None
        yy = CP.dense32(y) if y is not None else None
        dx = _mem.empty(dy.shape, dtype=torch.float32)
        CP.lib().unary_bwd(UNARY[op], CP.p(xx), CP.p(yy), dy.data_ptr(), dx.data_ptr(), dy.numel(), float(alpha))
        return dx
    xf = x.float() if x is not None else None
    yf = y.float() if y is not None else None
    g = dy.float()
    if op == "relu":
        r = g * (xf > 0)
    elif op == "sigmoid":
        r = g * yf * (1 - yf)
    elif op == "tanh":
        r = g * (1 - yf * yf)
    elif op == "stanh":
        r = g * (0.66666667 * 1.7159047 - 0.66666667 / 1.7159047 * yf * yf)
    elif op in ("gelu", "gelu_tanh"):
        with torch.enable_grad():
            xx = xf.detach().requires_grad_(True)
            out = F.gelu(xx, approximate="tanh" if op == "gelu_tanh" else "none")
            (r,) = torch.autograd.grad(out, xx, g)
    elif op in ("identity", "adds"):
        r = g
    elif op == "softplus":
        r = g * torch.sigmoid(xf)
    elif op == "square":
        r = g * 2 * xf
    elif op == "abs":
        r = g * torch.sign(xf)
    elif op == "exp":
        r = g * yf
    elif op == "leakyrelu":
        r = torch.where(xf > 0, g, alpha * g)
    elif op == "elu":
        r = torch.where(xf > 0, g, g * (yf + alpha))
    elif op == "selu":
        l, a = 1.0507009873554805, 1.6732632423543772
        r = torch.where(xf > 0, l * g, g * (yf + l * a))
    elif op == "sqrt":
        r = g * 0.5 / yf
    elif op == "neg":
        r = -g
    elif op == "reciprocal":
        r = -g * yf * yf
    elif op == "log":
        r = g / xf
    elif op in ("sign", "ceil", "floor", "round"):
        r = torch.zeros_like(g)
    elif op == "erf":
        r = g * 1.1283791671 * torch.exp(-xf * xf)
    elif op == "cos":
        r = -g * torch.sin(xf)
    elif op == "sin":
        r = g * torch.cos(xf)
    elif op == "tan":
        r = g * (1 + yf * yf)
    elif op == "cosh":
        r = g * torch.sinh(xf)
    elif op == "sinh":
        r = g * torch.cosh(xf)
    elif op == "acos":
        r = -g * torch.rsqrt(1 - xf * xf)
    elif op == "asin":
        r = g * torch.rsqrt(1 - xf * xf)
    elif op == "atan":
        r = g / (1 + xf * xf)
    elif op == "acosh":
        r = g * torch.rsqrt(xf * xf - 1)
    elif op == "asinh":
        r = g * torch.rsqrt(xf * xf + 1)
    elif op == "atanh":
        r = g / (1 - xf * xf)
    elif op == "softsign":
        r = g / (1 + xf.abs()) ** 2
    elif op == "scale":
        r = g * alpha
    elif op == "rsqrt":
        r = -0.5 * g * yf ** 3
    elif op == "pows":
        r = g * alpha * torch.pow(xf, alpha - 1)
    else:
        raise KeyError(op)
    return r.to(dy.dtype)


def add_act(a: torch.Tensor, b: torch.Tensor, alpha=1.0, beta=1.0, relu=False) -> torch.Tensor:
    if _native_ok(a, b) and _flat_ok(a) and a.dtype == b.dtype and a.shape == b.shape:
        a, b = _dense(a), _dense(b)
        if _same_layout(a, b):
            y = _like(a)
            N.lib().add_act(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), N.dt(a), alpha, beta, int(relu),
                            N.stream())
            return y
    if CP.ok(a, b) and a.shape == b.shape:
        r = G.binary("add", unary("scale", a, alpha) if alpha != 1.0 else a,
                     unary("scale", b, beta) if beta != 1.0 else b)
        return unary("relu", r) if relu else r
    r = alpha * a + beta * b
    return torch.relu(r) if relu else r


def relu_bwd_from_y(y: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    if _native_ok(y, dy) and _flat_ok(dy) and _same_layout(y, dy) and y.dtype == dy.dtype:
        dx = _like(dy)
        N.lib().relu_bwd_from_y(y.data_ptr(), dy.data_ptr(), dx.data_ptr(), dy.numel(), N.dt(dy), N.stream())
        return dx
    if CP.ok(y, dy) and y.shape == dy.shape:
        return unary_bwd("relu", y, None, dy)  # relu'(y) == relu'(x) for y = relu(x)
    return dy * (y > 0)


def cast(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    if x.dtype == dtype:
        return x
    if _native_ok(x) and _flat_ok(x) and dtype in (torch.float32, torch.bfloat16):
        x = _dense(x)
        y = _like(x, dtype)
        N.lib().cast(x.data_ptr(), N.dt(x), y.data_ptr(), N.dt(y), x.numel(), N.stream())
        return y
    return G.to(x, dtype)


def dropout_fwd(x: torch.Tensor, ratio: float, seed: int, offset: int,
                epoch: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """``epoch``: optional device int64 step counter mixed into the Philox key
    (keeps masks fresh across HIP-graph replays)."""
    pkeep = 1.0 - ratio
    if _native_ok(x) and x.dtype in (torch.float32, torch.bfloat16):
        x = _dense(x)
        y = _like(x)
        mask = _like(x, torch.uint8)
        N.lib().dropout_fwd(x.data_ptr(), y.data_ptr(), mask.data_ptr(), x.numel(), N.dt(x), pkeep, seed, offset,
                            N.ptr(epoch), N.stream())
        return y, mask
    _no_native("dropout_fwd", x)
    if CP.lib() is not None and not x.is_cuda:
        # the GPU kernels' Philox stream on the host (bit-identical masks); the
        # oracle applies the same mask with PyTorch arithmetic
        xc = CP.dense32(x)
        y = _mem.empty(x.shape, dtype=torch.float32)
        mask = _mem.empty(x.shape, dtype=torch.uint8)
        CP.lib().dropout_fwd(xc.data_ptr(), y.data_ptr(), mask.data_ptr(), xc.numel(), pkeep, int(seed), int(offset))
        if CP.ok(x):
            return y, mask
        return x * mask.to(x.dtype) / pkeep, mask
    g = torch.Generator(device=x.device).manual_seed(int(seed + offset) & 0x7FFFFFFFFFFFFFFF)
    mask = (torch.rand(x.shape, generator=g, device=x.device) < pkeep).to(torch.uint8)
    return x * mask.to(x.dtype) / pkeep, mask


def dropout_bwd(dy: torch.Tensor, mask: torch.Tensor, ratio: float) -> torch.Tensor:
    pkeep = 1.0 - ratio
    if _native_ok(dy) and dy.dtype in (torch.float32, torch.bfloat16):
        dy = _dense(dy)
        if not _same_layout(dy, mask):
            dy = G.contiguous(dy, torch.channels_last if N.is_cl(mask) and mask.dim() == 4 else torch.contiguous_format)
        dx = _like(dy)
        N.lib().dropout_bwd(dy.data_ptr(), mask.data_ptr(), dx.data_ptr(), dy.numel(), N.dt(dy), pkeep, N.stream())
        return dx
    _no_native("dropout_bwd", dy)
    if CP.ok(dy) and mask.dtype == torch.uint8 and mask.shape == dy.shape:
        dy, m = CP.dense32(dy), G.contiguous(mask)
        dx = _mem.empty(dy.shape, dtype=torch.float32)
        CP.lib().dropout_bwd(dy.data_ptr(), m.data_ptr(), dx.data_ptr(), dy.numel(), pkeep)
        return dx
    return dy * mask.to(dy.dtype) / pkeep


# ----------------------------------------------------------------------------
# softmax / losses / layernorm
# ----------------------------------------------------------------------------
def softmax(x: torch.Tensor, axis: int = -1, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """Row softmax over ``axis``; ``out_dtype`` (fp32 / bf16, default x's)
    lets fp32 scores come out as bf16 probabilities in the same pass."""
    axis = axis % x.dim()
    od = out_dtype or x.dtype
    if _native_ok(x) and x.dtype in (torch.float32, torch.bfloat16) and od in (torch.float32, torch.bfloat16):
        if axis != x.dim() - 1:  # softmax over a middle axis: move it last (native copies)
            y = softmax(G.contiguous(x.movedim(axis, -1)), -1, od)
            return G.contiguous(y.movedim(-1, axis))
        x = G.contiguous(x)
        C = x.shape[-1]
        if C <= 1024:  # short rows: one wave per row
            y = _mem.empty(x.shape, dtype=od, device=x.device)
            N.lib().softmax_rows(x.data_ptr(), y.data_ptr(), x.numel() // C, C, N.dt(x), N.dt(y), N.stream())
            return y
        if C > 16384:
            raise NotImplementedError(f"softmax: rows longer than 16384 ({C})")
        y = _mem.empty_like(x)
        N.lib().softmax_fwd(x.data_ptr(), y.data_ptr(), x.numel() // C, C, N.dt(x), int(x.dtype == torch.float32),
                            N.stream())
        return y if od == x.dtype else cast(y, od)
    _no_native("softmax", x)
    if CP.ok(x) and od == torch.float32:
        if axis != x.dim() - 1:
            return G.contiguous(softmax(G.contiguous(x.movedim(axis, -1)), -1, od).movedim(-1, axis))
        x = CP.dense32(x)
        y = _mem.empty(x.shape, dtype=torch.float32)
        n = x.shape[-1] if x.dim() else 1
        if y.numel():
            CP.lib().softmax(x.data_ptr(), y.data_ptr(), x.numel() // n, n)
        return y
    return torch.softmax(x.float(), dim=axis).to(od)


def softmax_bwd(y: torch.Tensor, dy: torch.Tensor, axis: int = -1) -> torch.Tensor:
    axis = axis % y.dim()
    if _native_ok(y, dy) and y.dtype in (torch.float32, torch.bfloat16):
        if axis != y.dim() - 1:
            g = softmax_bwd(G.contiguous(y.movedim(axis, -1)), G.contiguous(dy.movedim(axis, -1)), -1)
            return G.contiguous(g.movedim(-1, axis))
        y = G.contiguous(y)
        dy = G.contiguous(G.to(dy, y.dtype))
        C = y.shape[-1]
        dx = _mem.empty_like(dy)
        N.lib().softmax_bwd(y.data_ptr(), dy.data_ptr(), dx.data_ptr(), y.numel() // C, C, N.dt(y), N.stream())
        return dx
    _no_native("softmax_bwd", y, dy)
    if CP.ok(y, dy):
        if axis != y.dim() - 1:
            g = softmax_bwd(G.contiguous(y.movedim(axis, -1)), G.contiguous(dy.movedim(axis, -1)), -1)
            return G.contiguous(g.movedim(-1, axis))
        y, dy = CP.dense32(y), CP.dense32(dy)
        dx = _mem.empty(y.shape, dtype=torch.float32)
        n = y.shape[-1] if y.dim() else 1
        if dx.numel():
            CP.lib().softmax_bwd(y.data_ptr(), dy.data_ptr(), dx.data_ptr(), y.numel() // n, n)
        return dx
    yf, gf = y.float(), dy.float()
    return (yf * (gf - (gf * yf).sum(dim=axis, keepdim=True))).to(dy.dtype)


def softmax_xent(x: torch.Tensor, target: torch.Tensor, topk: int = 1, grad_scale: Optional[float] = None,
                 need_grad: bool = True):
    """Fused softmax + cross entropy.  target: int class ids [B] or a [B, C]
    probability matrix.  Returns (loss_per_row fp32 [B], correct fp32 [B],
    dx (p - t) * grad_scale or None).  grad_scale defaults to 1/B."""
    x2 = x.reshape(-1, x.shape[-1])
    B, C = x2.shape
    gs = (1.0 / B) if grad_scale is None else grad_scale
    soft = target.dim() > 1 and target.shape[-1] == C and target.is_floating_point()
    if _native_ok(x) and x2.dtype in (torch.float32, torch.bfloat16) and C <= 16384:
        x2 = G.contiguous(x2)
        loss = _mem.empty(B, dtype=torch.float32, device=x.device)
        correct = _mem.empty(B, dtype=torch.float32, device=x.device)
        dx = _mem.empty_like(x2) if need_grad else None
        if soft:
            t = G.contiguous(G.to(G.reshape(target, (B, C)), torch.float32))
            lab = None
        else:
            lab = G.contiguous(G.to(G.reshape(target, (B,)), torch.int32))
            t = None
        N.lib().softmax_xent(x2.data_ptr(), N.ptr(lab), N.ptr(t), loss.data_ptr(), correct.data_ptr(), N.ptr(dx), B,
                             C, N.dt(x2), topk, gs, N.stream())
        return loss, correct, (dx.reshape(x.shape) if dx is not None else None)
    _no_native("softmax_xent", x)
    if CP.ok(x2) and (not soft or target.dtype == torch.float32):
        x2 = CP.dense32(x2)
        loss = _mem.empty(B, dtype=torch.float32)
        correct = _mem.empty(B, dtype=torch.float32)
        dx = _mem.empty(x2.shape, dtype=torch.float32) if need_grad else None
        if soft:
            t, lab, l64 = CP.dense32(G.reshape(target, (B, C))), None, 0
        else:
            lab = G.contiguous(G.reshape(target, (B,)))
            if lab.dtype not in (torch.int32, torch.int64):
                lab = G.to(lab, torch.int32)
            t, l64 = None, int(lab.dtype == torch.int64)
        CP.lib().softmax_xent(x2.data_ptr(), CP.p(lab), l64, CP.p(t), loss.data_ptr(), correct.data_ptr(), CP.p(dx), B, C,
                             int(topk), float(gs))
        return loss, correct, (dx.reshape(x.shape) if dx is not None else None)
    xf = x2.float()
    lse = torch.logsumexp(xf, dim=1)
    if soft:
        t = target.reshape(B, C).float()
        loss = (t * (lse[:, None] - xf)).sum(1)
        correct = torch.zeros(B, dtype=torch.float32, device=x.device)
        dx = (torch.softmax(xf, 1) * t.sum(1, keepdim=True) - t) * gs if need_grad else None
    else:
        lab = target.reshape(B).long()
        xl = xf.gather(1, lab[:, None])[:, 0]
        loss = lse - xl
        rank = (xf > xl[:, None]).sum(1)
        correct = (rank < topk).float()
        if need_grad:
            p = torch.softmax(xf, 1)
            p[torch.arange(B, device=x.device), lab] -= 1.0
            dx = p * gs
        else:
            dx = None
    return loss, correct, (dx.to(x.dtype).reshape(x.shape) if dx is not None else None)


def layernorm_fwd(x: torch.Tensor, g: Optional[torch.Tensor], b: Optional[torch.Tensor], eps: float = 1e-5):
    D = x.shape[-1]
    if _native_ok(x) and x.dtype in (torch.float32, torch.bfloat16):
        x = G.contiguous(x)
        R = x.numel() // D
        y = _mem.empty_like(x)
        mean = _mem.empty(R, dtype=torch.float32, device=x.device)
        rstd = _mem.empty(R, dtype=torch.float32, device=x.device)
        gg = G.contiguous(G.to(g, torch.float32)) if g is not None else None
        bb = G.contiguous(G.to(b, torch.float32)) if b is not None else None
        N.lib().layernorm_fwd(x.data_ptr(), N.ptr(gg), N.ptr(bb), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), R,
                              D, N.dt(x), eps, N.stream())
        return y, mean, rstd
    _no_native("layernorm_fwd", x)
    if CP.ok(x, g, b):
        x = CP.dense32(x)
        R = x.numel() // D
        y = _mem.empty(x.shape, dtype=torch.float32)
        mean = _mem.empty(R, dtype=torch.float32)
        rstd = _mem.empty(R, dtype=torch.float32)
        gg = CP.dense32(g) if g is not None else None
        bb = CP.dense32(b) if b is not None else None
        CP.lib().layernorm_fwd(x.data_ptr(), CP.p(gg), CP.p(bb), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), R, D,
                               float(eps))
        return y, mean, rstd
    xf = x.float().reshape(-1, D)
    mean = xf.mean(1)
    rstd = torch.rsqrt(xf.var(1, unbiased=False) + eps)
    y = (xf - mean[:, None]) * rstd[:, None]
    if g is not None:
        y = y * g.float()
    if b is not None:
        y = y + b.float()
    return y.to(x.dtype).reshape(x.shape), mean, rstd


def drop_add_ln_ok(x: torch.Tensor, a: torch.Tensor) -> bool:
    """The fused y = LayerNorm(x + dropout(a)) kernels apply (native, same
    shape and dtype, last dim % 8 == 0 and <= 2048)."""
    D = x.shape[-1] if x.dim() else 0
    return (_native_ok(x, a) and x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and a.dtype == x.dtype
            and tuple(a.shape) == tuple(x.shape) and D % 8 == 0 and 0 < D <= 2048)


def drop_add_layernorm_fwd(x, a, g, b, eps: float, ratio: float, seed: int = 0, offset: int = 0, epoch=None):
    """y = LayerNorm(s), s = x + dropout(a), in one pass (native; see
    drop_add_ln_ok).  The mask is the dropout kernel's own Philox stream for
    (seed, offset), so the result is bitwise the dropout -> add -> LayerNorm
    chain's.  Returns (y, s, mask or None, mean, rstd)."""
    D = x.shape[-1]
    R = x.numel() // D
    x, a = G.contiguous(x), G.contiguous(a)
    s = _mem.empty_like(x)
    y = _mem.empty_like(x)
    mean = _mem.empty(R, dtype=torch.float32, device=x.device)
    rstd = _mem.empty(R, dtype=torch.float32, device=x.device)
    mask = _mem.empty(x.shape, dtype=torch.uint8, device=x.device) if ratio > 0 else None
    gg = G.contiguous(G.to(g, torch.float32)) if g is not None else None
    bb = G.contiguous(G.to(b, torch.float32)) if b is not None else None
    N.lib().drop_add_ln_fwd(x.data_ptr(), a.data_ptr(), N.ptr(gg), N.ptr(bb), s.data_ptr(), N.ptr(mask), y.data_ptr(),
                            mean.data_ptr(), rstd.data_ptr(), R, D, N.dt(x), eps, 1.0 - ratio if ratio > 0 else 1.0,
                            seed, offset, N.ptr(epoch), N.stream())
    return y, s, mask, mean, rstd


def drop_add_layernorm_bwd(s, dy, g, mean, rstd, mask, ratio: float, dg_acc=None, db_acc=None, cs_acc=None):
    """Backward of drop_add_layernorm_fwd in one pass: (ds, da, dg, db, cs) --
    ds the gradient of x (and of s), da = ds * mask / (1 - ratio) that of a,
    cs the column sums of da (fp32 [D]: the bias gradient of the Linear that
    produced a); dg / db / cs accumulate into the *_acc views when given
    (``cs_acc``: that Linear's bias-gradient view itself)."""
    D = s.shape[-1]
    R = s.numel() // D
    L = N.lib()
    dy = G.contiguous(G.to(dy, s.dtype))
    ds, da = _mem.empty_like(s), _mem.empty_like(s)

    def _acc(t):
        ok = t is not None and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == D and t.is_cuda
        return t if ok else _zeros32(D, s.device)

    dg, db = (_acc(dg_acc), _acc(db_acc)) if g is not None else (None, None)
    cs = _acc(cs_acc)
    ws = _mem.empty(L.layernorm_bwd_ws(R, D) * 3 // 2, dtype=torch.float32, device=s.device)
    gg = G.contiguous(G.to(g, torch.float32)) if g is not None else None
    L.drop_add_ln_bwd(s.data_ptr(), dy.data_ptr(), N.ptr(gg), mean.data_ptr(), rstd.data_ptr(), N.ptr(mask),
                      1.0 - ratio if mask is not None else 1.0, ds.data_ptr(), da.data_ptr(), N.ptr(dg), N.ptr(db),
                      cs.data_ptr(), ws.data_ptr(), R, D, N.dt(s), N.stream())
    return ds, da, dg, db, cs


LNB_V2 = os.environ.get("SINGA_AMD_LNB_V2", "1") != "0"  # (A/B switch: the v1 single-kernel backward)


def layernorm_bwd(x, dy, g, mean, rstd, dg_acc=None, db_acc=None):
    """Returns (dx, dg, db).  ``dg_acc`` / ``db_acc``: fp32 [D] gradient
    buffers (the parameters' flat-store views) the kernel ACCUMULATES into
    directly -- returned as dg / db (no zeroed temporaries, no extra adds)."""
    D = x.shape[-1]
    R = x.numel() // D

    def _acc_ok(t):
        return t is not None and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == D and t.is_cuda

    if _native_ok(x, dy) and x.dtype in (torch.float32, torch.bfloat16):
        x = G.contiguous(x)
        dy = G.contiguous(G.to(dy, x.dtype))
        dx = _mem.empty_like(x)
        dg = db = None
        if g is not None:
            dg = dg_acc if _acc_ok(dg_acc) else G.zeros((D,), torch.float32, x.device)
            db = db_acc if _acc_ok(db_acc) else G.zeros((D,), torch.float32, x.device)
        gg = G.contiguous(G.to(g, torch.float32)) if g is not None else None
        L = N.lib()
        nws = L.layernorm_bwd_ws(R, D) if LNB_V2 else 0
        if nws:  # pipelined rows, per-workgroup partial dgamma / dbeta rows folded by a second kernel
            ws = _mem.empty(nws, dtype=torch.float32, device=x.device) if dg is not None else None
            L.layernorm_bwd_v2(x.data_ptr(), dy.data_ptr(), N.ptr(gg), mean.data_ptr(), rstd.data_ptr(),
                               dx.data_ptr(), N.ptr(dg), N.ptr(db), N.ptr(ws), R, D, N.dt(x), N.stream())
        else:
            L.layernorm_bwd(x.data_ptr(), dy.data_ptr(), N.ptr(gg), mean.data_ptr(), rstd.data_ptr(),
                            dx.data_ptr(), N.ptr(dg), N.ptr(db), R, D, N.dt(x), N.stream())
        return dx, dg, db
    _no_native("layernorm_bwd", x, dy)
    if CP.ok(x, dy, g):
        x, dy = CP.dense32(x), CP.dense32(dy)
        dx = _mem.empty(x.shape, dtype=torch.float32)
        dg = db = None
        if g is not None:
            dg = dg_acc if (dg_acc is not None and CP.ok(dg_acc) and dg_acc.is_contiguous() and dg_acc.numel() == D) \
                else G.zeros((D,), torch.float32, x.device)
            db = db_acc if (db_acc is not None and CP.ok(db_acc) and db_acc.is_contiguous() and db_acc.numel() == D) \
                else G.zeros((D,), torch.float32, x.device)
        gg = CP.dense32(g) if g is not None else None
        CP.lib().layernorm_bwd(x.data_ptr(), dy.data_ptr(), CP.p(gg), CP.dense32(mean).data_ptr(),
                               CP.dense32(rstd).data_ptr(), dx.data_ptr(), CP.p(dg), CP.p(db), R, D)
        if dg is not None and dg_acc is not None and dg is not dg_acc:
            dg = G.binary("add", dg_acc, G.reshape(dg, dg_acc.shape), out=dg_acc)
            db = G.binary("add", db_acc, G.reshape(db, db_acc.shape), out=db_acc)
        return dx, dg, db
    xf = x.float().reshape(R, D)
    gy = dy.float().reshape(R, D)
    xh = (xf - mean[:, None]) * rstd[:, None]
    dg = (gy * xh).sum(0) if g is not None else None
    db = gy.sum(0) if g is not None else None
    gg = gy * g.float() if g is not None else gy
    a = gg.mean(1, keepdim=True)
    bsum = (gg * xh).mean(1, keepdim=True)
    dx = rstd[:, None] * (gg - a - xh * bsum)
    if dg is not None and dg_acc is not None:
        dg = dg_acc.add_(dg.reshape(dg_acc.shape))
    if db is not None and db_acc is not None:
        db = db_acc.add_(db.reshape(db_acc.shape))
    return dx.to(x.dtype).reshape(x.shape), dg, db


# ----------------------------------------------------------------------------
# GEMM
# ----------------------------------------------------------------------------
def _no_native(what: str, *ts) -> None:
    """GPU operands must run on a hand-written kernel: raise instead of
    silently handing a device tensor to a PyTorch/vendor kernel.
    (native._TORCH_ORACLE_FOR_TESTS -- a test-only hook -- re-enables the PyTorch path.)"""
    if N.force_native() and any(t is not None and t.is_cuda for t in ts):
        raise NotImplementedError(f"{what}: no native gfx950 kernel for this case "
                                  f"({[(tuple(t.shape), t.dtype) for t in ts if t is not None]})")


def _mat(t: torch.Tensor, trans: bool):
    """View a 2-D operand (or the last two dims of a 3-D one) as (tensor, ld,
    k_outer) where the logical op(t) is [rows][K]: dense row-major, or
    column-major (a transposed view) taken as is; other strides are copied."""
    r, c = t.shape[-2], t.shape[-1]
    s0, s1 = t.stride(-2), t.stride(-1)
    if (s1 == 1 or c == 1) and (r == 1 or s0 >= c):  # row-major: t[i][j] at i*ld + j
        return t, (s0 if r > 1 else max(c, 1)), bool(trans)
    if (s0 == 1 or r == 1) and (c == 1 or s1 >= r):  # column-major: t[i][j] at j*ld + i
        return t, (s1 if c > 1 else max(r, 1)), not trans
    t = G.contiguous(t)
    return t, max(c, 1), bool(trans)


def _igemm_ok(a, lda, ako, b, ldb, bko, M, Nn, K, sa, sb) -> bool:
    """The tuned bf16 kernel (igemm.hip: 16-byte LDS-DMA chunks of 8
    elements) takes the problem: K-major operands need K % 8, K-outer ones
    rows % 8, every leading dimension / batch stride % 8, 16-byte bases."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        return False
    for t, ld, ko, rows, st in ((a, lda, ako, M, sa), (b, ldb, bko, Nn, sb)):
        if ld % 8 or st % 8 or t.data_ptr() % 16:
            return False
        if (ko and rows % 8) or (not ko and K % 8):
            return False
        if t.numel() * 2 >= (1 << 31):
            return False
    return True


GEMM_ACT = {"relu": 1, "sigmoid": 2, "tanh": 3, "stanh": 4, "gelu": 5, "gelu_tanh": 6}  # epilogue Act codes
ACT_XFORM = {"gelu", "gelu_tanh"}  # derivative from the activation's input z (the others: from its output)


def gemm(a: torch.Tensor, b: torch.Tensor, ta: bool = False, tb: bool = False, out: Optional[torch.Tensor] = None,
         out_dtype: Optional[torch.dtype] = None, alpha: float = 1.0, beta: float = 0.0,
         bias: Optional[torch.Tensor] = None, relu: bool = False, accumulate: bool = False,
         colsum_b: Optional[torch.Tensor] = None, act: Optional[str] = None,
         act_grad: Optional[Tuple[str, torch.Tensor]] = None, act_aux: Optional[torch.Tensor] = None,
         colsum_c: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C = alpha * op(a) @ op(b) (+ beta * C) (+ bias[n]) (ReLU), op(t) = t.T if
    the flag is set.  2-D or batched 3-D operands (equal batch, or one side
    2-D and shared).  ``accumulate``: C (fp32 ``out``) += alpha * op(a) op(b)
    (split-K atomics).  ``colsum_b`` (fp32 [N], 2-D operands): += the column
    sums of op(b) -- a weight-gradient GEMM's bias gradient, summed by the
    generic kernel from the tiles it stages anyway.  ``act`` (relu / sigmoid
    / tanh / stanh / gelu / gelu_tanh): activation of the output, with the
    pre-activation written to ``act_aux`` when given; ``act_grad`` = (act, t):
    C *= act'(t), t that activation's output (or, for the gelus, its input)
    laid out like C -- a data-gradient GEMM taking its producer's activation
    backward.  Both run in the GEMM epilogues on the GPU (rounded exactly as
    the separate elementwise kernels would); the host applies them in a
    separate pass.  ``colsum_c`` (fp32 [N], with ``act_grad``): += the column
    sums of the final C -- that producer's bias gradient -- summed in the
    same epilogue where the tuned kernel takes the call, else by a separate
    pass.  On the
    GPU: bf16 operands of aligned shapes run the tuned MFMA kernel,
    everything else (fp32 -- exact f32 MFMA -- and ragged bf16) the generic
    one; there is no vendor-BLAS path."""
    if colsum_b is not None and (a.dim() != 2 or b.dim() != 2):
        raise ValueError("gemm: colsum_b needs 2-D operands")
    if colsum_c is not None:
        if act_grad is None or a.dim() != 2 or b.dim() != 2:
            raise ValueError("gemm: colsum_c needs act_grad and 2-D operands")
        if colsum_c.dtype != torch.float32 or not colsum_c.is_contiguous():
            raise ValueError("gemm: colsum_c must be a dense fp32 [N] tensor")
    if act == "relu" and act_grad is None and act_aux is None:
        act, relu = None, True
    if act is not None or act_grad is not None:
        if act is not None and act not in GEMM_ACT or act_grad is not None and act_grad[0] not in GEMM_ACT:
            raise ValueError(f"gemm: unsupported fused activation {act or act_grad[0]}")
        if relu or accumulate or act is not None and act_grad is not None:
            raise ValueError("gemm: act / act_grad exclude each other, relu and accumulate")
        dt = out.dtype if out is not None else (out_dtype or a.dtype)
        fused = (a.is_cuda and N.available() and a.dtype == b.dtype == dt and dt in (torch.float32, torch.bfloat16)
                 and beta == 0.0)
        if not fused:
            c = _gemm_act_unfused(a, b, ta, tb, out, out_dtype, alpha, beta, bias, colsum_b, act, act_grad, act_aux)
            if colsum_c is not None:
                _colsum_into(c, colsum_c)
            return c
        for t in ((act_grad[1] if act_grad is not None else None), act_aux):
            if t is not None and (t.dtype != dt or not t.is_contiguous()):
                raise ValueError("gemm: act_grad / act_aux tensors must be dense and of the output dtype")
    if a.dim() == 2 and b.dim() == 2:
        batch = 1
    elif a.dim() == 3 and b.dim() == 2 and not ta and a.is_contiguous() and out is None:
        Bt = a.shape[0]
        ag = (act_grad[0], act_grad[1].reshape(-1, act_grad[1].shape[-1])) if act_grad is not None else None
        aux = act_aux.reshape(-1, act_aux.shape[-1]) if act_aux is not None else None
        c = gemm(a.reshape(-1, a.shape[-1]), b, False, tb, None, out_dtype, alpha, beta, bias, relu, act=act,
                 act_grad=ag, act_aux=aux)
        return c.reshape(Bt, a.shape[1], c.shape[-1])
    elif a.dim() == 3 or b.dim() == 3:
        batch = a.shape[0] if a.dim() == 3 else b.shape[0]
        if (a.dim() == 3 and a.shape[0] != batch) or (b.dim() == 3 and b.shape[0] != batch):
            raise ValueError(f"gemm: batch mismatch {tuple(a.shape)} x {tuple(b.shape)}")
    else:
        raise ValueError(f"gemm: expected 2-D / 3-D operands, got {tuple(a.shape)} x {tuple(b.shape)}")
    M, K = (a.shape[-1], a.shape[-2]) if ta else (a.shape[-2], a.shape[-1])
    Kb, Nn = (b.shape[-1], b.shape[-2]) if tb else (b.shape[-2], b.shape[-1])
    if K != Kb:
        raise ValueError(f"gemm: inner dims differ {tuple(a.shape)} x {tuple(b.shape)} (ta={ta}, tb={tb})")
    lead = (batch,) if batch > 1 or a.dim() == 3 or b.dim() == 3 else ()
    if out is None:
        od = out_dtype or (torch.float32 if accumulate else a.dtype)
        out = G.zeros(lead + (M, Nn), od, a.device) if accumulate else _mem.empty(lead + (M, Nn), dtype=od,
                                                                                      device=a.device)
    if (not a.is_cuda and CP.ok(a, b, bias) and out.dtype == torch.float32 and out.is_contiguous()
            and (bias is None or bias.numel() == Nn)):
        if M == 0 or Nn == 0:
            return out
        a, lda, ako = _mat(a, ta)
        b, ldb, bko = _mat(b, tb)
        sa = a.stride(0) if a.dim() == 3 else 0
        sb = b.stride(0) if b.dim() == 3 else 0
        sc = M * Nn if out.dim() == 3 else 0
        bb = CP.dense32(bias).reshape(-1) if bias is not None else None
        if batch > 1 and (bb is not None or relu):
            for i in range(batch):
                gemm(a[i] if a.dim() == 3 else a, b[i] if b.dim() == 3 else b, ta, tb, out[i], None, alpha,
                     1.0 if accumulate else beta, bias, relu)
            return out
        CP.gemm(a, lda, ako, b, ldb, not bko, out, M, Nn, K, alpha, 1.0 if accumulate else beta, bb, relu, batch, sa,
                sb, sc)
        if colsum_b is not None:
            _colsum_opb(b, tb, colsum_b)
        return out
    if not (_native_ok(a, b) and a.is_cuda):
        if a.is_cuda:
            _no_native("gemm", a, b)
        aa = a.float().transpose(-1, -2) if ta else a.float()
        bb = b.float().transpose(-1, -2) if tb else b.float()
        if colsum_b is not None:
            colsum_b.add_(bb.sum(0))
        r = alpha * torch.matmul(aa, bb)
        if accumulate:
            return out.add_(r.reshape(out.shape))
        if beta != 0.0:
            r = r + beta * out.float()
        if bias is not None:
            r = r + bias.float()
        if relu:
            r = torch.relu(r)
        out.copy_(r.reshape(out.shape))
        return out
    if a.dtype != b.dtype:  # mixed operands: the wider type
        a, b = cast(a, torch.float32), cast(b, torch.float32)
    if not out.is_contiguous() or out.dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("gemm: output must be a dense fp32/bf16 tensor")
    if accumulate and out.dtype != torch.float32:
        raise ValueError("gemm: accumulation needs an fp32 output")
    if M == 0 or Nn == 0:
        return out
    a, lda, ako = _mat(a, ta)
    b, ldb, bko = _mat(b, tb)
    bko = not bko  # B(n, k) convention of the kernels: k_outer == B stored [K][N]
    sa = a.stride(0) if a.dim() == 3 else 0
    sb = b.stride(0) if b.dim() == 3 else 0
    sc = M * Nn if out.dim() == 3 else 0
    bb = G.contiguous(G.to(bias, torch.float32)).reshape(-1) if bias is not None else None
    mode = 2 if accumulate else (0 if out.dtype == torch.bfloat16 else 1)
    L = N.lib()
    code = GEMM_ACT[act] if act is not None else int(relu)
    ab, ax = (GEMM_ACT[act_grad[0]], act_grad[1]) if act_grad is not None else (0, None)
    for t in (ax, act_aux):
        if t is not None and tuple(t.shape) != tuple(out.shape):
            raise ValueError(f"gemm: act_grad / act_aux {tuple(t.shape)} != C {tuple(out.shape)}")
    if _igemm_ok(a, lda, ako, b, ldb, bko, M, Nn, K, sa, sb) and (mode == 2 or sc % 8 == 0) and K > 0:
        if act is not None or act_grad is not None:
            # fused activation: the tuned kernel's LDS-staged epilogue (bf16
            # output, batch 1, N % 8), else the generic kernel below
            if colsum_c is not None and colsum_c.numel() != Nn:
                raise ValueError(f"gemm: colsum_c has {colsum_c.numel()} entries, C has {Nn} columns")
            if mode == 0 and batch == 1 and colsum_b is None and L.gemm_act(
                    a.data_ptr(), lda, int(ako), b.data_ptr(), ldb, int(bko), out.data_ptr(), Nn, M, Nn, K, alpha,
                    N.ptr(bb), batch, sa, sb, sc, code if act is not None else 0, N.ptr(act_aux), ab, N.ptr(ax),
                    N.ptr(colsum_c), N.stream()):
                return out
        else:
            L.gemm(a.data_ptr(), lda, int(ako), b.data_ptr(), ldb, int(bko), out.data_ptr(), Nn, M, Nn, K, alpha,
                   beta, N.ptr(bb), int(relu), mode, 0 if mode == 2 else 1, batch, sa, sb, sc, N.stream())
            if colsum_b is not None:
                _colsum_opb(b, not bko, colsum_b)
            return out
    if a.dtype not in (torch.float32, torch.bfloat16):
        _no_native(f"gemm ({a.dtype})", a)
    cs = 0
    if colsum_b is not None:
        if colsum_b.dtype != torch.float32 or not colsum_b.is_contiguous() or colsum_b.numel() != Nn:
            raise ValueError("gemm: colsum_b must be a dense fp32 [N] tensor")
        cs = colsum_b.data_ptr()
    if act in ACT_XFORM or act_grad is not None and act_grad[0] in ACT_XFORM:
        # (the generic kernel's epilogue carries only the y-form activations)
        c = _gemm_act_unfused(a, b, ta, tb, out, None, alpha, beta, bias, colsum_b, act, act_grad, act_aux)
        if colsum_c is not None:
            _colsum_into(c, colsum_c)
        return c
    L.ggemm(0 if a.dtype == torch.float32 else 1, a.data_ptr(), lda, int(ako), sa, b.data_ptr(), ldb, int(bko), sb,
            out.data_ptr(), Nn, sc, M, Nn, K, alpha, beta, N.ptr(bb), code, mode, 0, batch, cs, ab, N.ptr(ax),
            N.ptr(act_aux), N.stream())
    if colsum_c is not None:
        _colsum_into(out, colsum_c)
    return out


def _colsum_into(c: torch.Tensor, out: torch.Tensor) -> None:
    """out += column sums of the 2-D C (the separate pass behind gemm's colsum_c)."""
    if c.is_cuda:
        colsum(G.contiguous(c), out=out)
    else:
        out.add_(c.float().sum(0))


def _gemm_act_unfused(a, b, ta, tb, out, out_dtype, alpha, beta, bias, colsum_b, act, act_grad, act_aux):
    """gemm() followed by the activation (or its derivative) as a separate
    elementwise pass: the host path, and shapes no fused epilogue takes."""
    c = gemm(a, b, ta, tb, out, out_dtype, alpha, beta, bias, False, False, colsum_b)
    r = c
    if act is not None:
        if act_aux is not None:
            G.copy_(act_aux, c)
        r = unary(act, r)
    if act_grad is not None:
        k, t = act_grad
        if k == "relu":
            r = relu_bwd_from_y(t, r)
        else:
            r = unary_bwd(k, t, None, r) if k in ACT_XFORM else unary_bwd(k, None, t, r)
    if r is not c:
        G.copy_(c, r)
    return c


def _colsum_opb(b: torch.Tensor, tb: bool, out: torch.Tensor) -> None:
    """out += column sums of op(b) (op = transpose if ``tb``): the separate
    pass for the GEMM paths that do not fuse it."""
    if tb:
        out_, _ = colsum(G.contiguous(b.t()))
        G.binary("add", out, out_, out=out)
    else:
        colsum(G.contiguous(b), out=out)


def matmul(a: torch.Tensor, b: torch.Tensor, out_dtype: Optional[torch.dtype] = None,
           bias: Optional[torch.Tensor] = None, relu: bool = False, act: Optional[str] = None,
           act_aux: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C = a @ b for 2-D (or batched 3-D with equal batch) row-major operands.
    bf16 operands run on the MFMA kernel with fp32 accumulation; fp32
    operands on the exact-f32 MFMA kernel (``act``: fused output activation,
    see :func:`gemm`)."""
    if a.dim() > 3 or b.dim() > 3:  # flatten equal leading dims (torch.matmul broadcasting otherwise)
        lead = torch.broadcast_shapes(a.shape[:-2], b.shape[:-2])
        aa = G.reshape(a.expand(*lead, *a.shape[-2:]), (-1, *a.shape[-2:]))
        bb = G.reshape(b.expand(*lead, *b.shape[-2:]), (-1, *b.shape[-2:]))
        c = gemm(aa, bb, out_dtype=out_dtype or a.dtype, bias=bias, relu=relu, act=act, act_aux=act_aux)
        return c.reshape(*lead, c.shape[-2], c.shape[-1])
    if a.dim() == 3 and b.dim() == 3 and a.shape[0] != b.shape[0]:
        lead = torch.broadcast_shapes(a.shape[:1], b.shape[:1])
        a = a.expand(*lead, *a.shape[-2:])
        b = b.expand(*lead, *b.shape[-2:])
    return gemm(a, b, out_dtype=out_dtype or a.dtype, bias=bias, relu=relu, act=act, act_aux=act_aux)


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out_dtype=None, bias=None, relu=False, act_grad=None,
            colsum_c=None) -> torch.Tensor:
    """C = a @ b.T (both operands K-major: a [M,K], b [N,K]); ``act_grad`` / ``colsum_c`` as in :func:`gemm`."""
    return gemm(a, b, tb=True, out_dtype=out_dtype or a.dtype, bias=bias, relu=relu, act_grad=act_grad,
                colsum_c=colsum_c)


def gemm_tn_acc(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, beta: float = 1.0,
                colsum_b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out (fp32) = beta*out + a.T @ b with a [K,M], b [K,N] (weight-gradient
    shape: reduction over the batch dim).  Uses split-K atomics on GPU.
    ``colsum_b`` (fp32 [N]) += the column sums of b (the bias gradient), fused
    into the GEMM where the kernel supports it."""
    if out.is_cuda and N.available():
        if beta == 0.0:
            N.lib().zero(out.data_ptr(), out.numel() * out.element_size(), N.stream())
        elif beta != 1.0:
            G.binary("mul", out, beta, out=out)
        return gemm(a, b, ta=True, out=out, accumulate=True, colsum_b=colsum_b)
    if CP.ok(a, b, out) and out.is_contiguous():
        return gemm(a, b, ta=True, out=out, beta=beta, colsum_b=colsum_b)
    r = a.float().t() @ b.float()
    if colsum_b is not None:
        colsum_b.add_(b.float().sum(0))
    if beta == 0.0:
        out.copy_(r)
    else:
        out.mul_(beta).add_(r)
    return out


# ----------------------------------------------------------------------------
# convolution (NCHW logical, NHWC physical on GPU)
# ----------------------------------------------------------------------------
def conv_out_size(h, k, s, p, d=1):
    return (h + 2 * p - d * (k - 1) - 1) // s + 1


def _pad8(n: int) -> int:
    return (n + 7) // 8 * 8


def to_nhwc_bf16(x: torch.Tensor, cpad: Optional[int] = None) -> torch.Tensor:
    """NCHW-logical tensor -> bf16 channels_last, optionally zero-padding C."""
    Nn, C, H, W = x.shape
    cp = cpad or C
    if cp != C:
        if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.is_contiguous() and cp % 8 == 0:
            y = _mem.empty((Nn, cp, H, W), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
            fn = N.lib().nchw_to_nhwc_pad if x.dtype == torch.float32 else N.lib().nchw_to_nhwc_pad_bf16
            fn(x.data_ptr(), y.data_ptr(), Nn, C, H, W, cp, N.stream())
            return y
        y = _zeros_cl((Nn, cp, H, W), torch.bfloat16, x.device)
        G.copy_(y[:, :C], x)
        return y
    return G.to(x, torch.bfloat16, torch.channels_last)


def _nhwc(t: torch.Tensor, dt: torch.dtype) -> torch.Tensor:
    """Dense channels_last copy of a 4-D tensor in dtype dt (no copy if it already is)."""
    if t.dtype == dt and N.is_cl(t):
        return t
    if t.dtype == dt and t.is_contiguous() and t.dim() == 4 and t.shape[2] * t.shape[3] == 1:
        return t  # [N, C, 1, 1]: NCHW and NHWC memory are the same
    return G.to(t, dt, torch.channels_last)


def _gconv_dt(*ts) -> torch.dtype:
    return torch.float32 if any(t is not None and t.dtype == torch.float32 for t in ts) else torch.bfloat16


def _gconv_fwd(x, w, b, stride, padding, dilation, groups, out_dtype, relu):
    """Generic-kernel convolution (ggemm.hip): fp32 operands in exact f32
    MFMA (no downcast), or bf16 grouped / dilated / unpadded-channel convs."""
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    Nn, C, H, W = x.shape
    K, Cg, R, S = w.shape
    if C != Cg * groups or K % groups:
        raise ValueError(f"conv2d: input {tuple(x.shape)} / weight {tuple(w.shape)} / groups {groups} mismatch")
    Ho, Wo = conv_out_size(H, R, sh, ph, dh), conv_out_size(W, S, sw, pw, dw)
    dt = _gconv_dt(x, w)
    xc, wc = _nhwc(x, dt), _nhwc(w, dt)
    od = torch.bfloat16 if out_dtype == torch.bfloat16 else torch.float32
    y = _mem.empty((Nn, K, Ho, Wo), dtype=od, device=x.device, memory_format=torch.channels_last)
    bias = G.contiguous(G.to(b, torch.float32)) if b is not None else None
    N.lib().gconv_fwd(0 if dt == torch.float32 else 1, xc.data_ptr(), wc.data_ptr(), y.data_ptr(), N.ptr(bias), Nn,
                      H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, groups, int(relu),
                      0 if od == torch.bfloat16 else 1, N.stream())
    return y if y.dtype == out_dtype else cast(y, out_dtype)


def _db_ok(db_out, K):
    return db_out is not None and db_out.dtype == torch.float32 and db_out.is_contiguous() and db_out.numel() == K


def _gconv_bwd(x, w, dy, stride, padding, dilation, groups, need_dx, dw_out, need_db, dx_acc, db_out=None):
    sh, sw = stride
    ph, pw = padding
    dh, dw_ = dilation
    Nn, C, H, W = x.shape
    K, Cg, R, S = w.shape
    Ho, Wo = dy.shape[2], dy.shape[3]
    dt = _gconv_dt(x, w, dy)
    dtc = 0 if dt == torch.float32 else 1
    L = N.lib()
    xc, wc, dyc = _nhwc(x, dt), _nhwc(w, dt), _nhwc(dy, dt)
    dx = None
    if need_dx:
        od = x.dtype if x.dtype in (torch.float32, torch.bfloat16) else dt
        if (dx_acc is not None and dx_acc.dtype == od and tuple(dx_acc.shape) == tuple(x.shape) and N.is_cl(dx_acc)
                and dx_acc.is_contiguous(memory_format=torch.channels_last)):
            dx, beta = dx_acc, 1.0
        else:
            dx, beta = _mem.empty(x.shape, dtype=od, device=x.device, memory_format=torch.channels_last), 0.0
        L.gconv_dgrad(dtc, dyc.data_ptr(), wc.data_ptr(), dx.data_ptr(), Nn, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw,
                      dh, dw_, groups, 0 if od == torch.bfloat16 else 1, beta, N.stream())
        if beta == 0.0:
            dx._sg_fresh = True
    direct = dw_out is not None and dw_out.dtype == torch.float32 and N.is_cl(dw_out)
    target = dw_out if direct else _zeros_cl((K, Cg, R, S), torch.float32, x.device)
    L.gconv_wgrad(dtc, xc.data_ptr(), dyc.data_ptr(), target.data_ptr(), Nn, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw,
                  dh, dw_, groups, 0, N.stream())
    if direct:
        dwt = dw_out
    elif dw_out is not None:
        dwt = G.binary("add", dw_out, target, out=dw_out)
    else:
        dwt = target
    db = None
    if need_db:
        acc = _db_ok(db_out, K)
        db = colsum(dyc.permute(0, 2, 3, 1).reshape(-1, K), out=db_out.view(-1) if acc else None)[0]
        if db_out is not None and not acc:
            db = G.binary("add", db_out, G.reshape(db, db_out.shape), out=db_out)
    return dx, dwt, db


def conv2d_fwd(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], stride, padding, dilation=(1, 1),
               groups: int = 1, out_dtype: Optional[torch.dtype] = None, relu: bool = False,
               bn_stats: bool = False) -> torch.Tensor:
    """x [N,C,H,W], w [K,C/g,R,S] -> y [N,K,Ho,Wo] (channels_last on GPU).
    ``bn_stats``: the epilogue also sums per-channel (x, x^2) of the bf16
    output into a BatchNorm workspace attached as ``y._sg_bn_ws`` (the next
    BatchNorm skips its statistics pass)."""
    out_dtype = out_dtype or x.dtype
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    if _native_ok(x, w) and not (groups == 1 and x.dtype == torch.bfloat16):
        return _gconv_fwd(x, w, b, stride, padding, dilation, groups, out_dtype, relu)
    if _native_ok(x, w) and groups == 1:
        Nn, Cx, H, W = x.shape
        K, C, R, S = w.shape
        Ho, Wo = conv_out_size(H, R, sh, ph, dh), conv_out_size(W, S, sw, pw, dw)
        Cp, Kp = _pad8(C), _pad8(K)
        if Cx not in (C, Cp):
            raise ValueError(f"conv2d: input has {Cx} channels, weight expects {C}")
        xb = x if (x.dtype == torch.bfloat16 and N.is_cl(x) and Cx == Cp) else to_nhwc_bf16(x[:, :C], Cp)
        wb = w
        if Cp != C or Kp != K:
            wb = _zeros_cl((Kp, Cp, R, S), torch.bfloat16, w.device)
            G.copy_(wb[:K, :C], w)
        elif not (w.dtype == torch.bfloat16 and N.is_cl(w)):
            wb = G.to(w, torch.bfloat16, torch.channels_last)
        bias = None
        if b is not None:
            bias = G.contiguous(G.to(b, torch.float32))
            if Kp != K:
                bias = G.cat([bias, G.zeros((Kp - K,), torch.float32, bias.device)])
        od = torch.bfloat16 if out_dtype == torch.bfloat16 else torch.float32
        y = _mem.empty((Nn, Kp, Ho, Wo), dtype=od, device=x.device, memory_format=torch.channels_last)
        ws, rows = None, 0
        if (bn_stats and od == torch.bfloat16 and Kp == K and out_dtype == torch.bfloat16 and not relu
                and not _NO_BN_STATS):
            L = N.lib()
            rows = L.conv_stats_rows(Nn * Ho * Wo, K)
            if rows > 0:  # deterministic: every row written (plain stores); else 32 atomic slot rows (zeroed)
                ws = zeroed_ws(rows * 2 * K, x.device)
        N.lib().conv_fwd(xb.data_ptr(), wb.data_ptr(), y.data_ptr(), N.ptr(bias), Nn, H, W, Cp, Kp, R, S, Ho, Wo, sh,
                         sw, ph, pw, dh, dw, int(relu), 0 if od == torch.bfloat16 else 1, N.stream(), N.ptr(ws))
        if xb is not x:  # converted input (network entry): the backward's weight gradient can reuse it
            y._sg_xconv = xb
        if ws is not None:
            y._sg_bn_ws = (ws, rows)
        if Kp != K:
            y = G.contiguous(y[:, :K], torch.channels_last)
        return y if y.dtype == out_dtype else cast(y, out_dtype)
    _no_native("conv2d_fwd", x, w)
    if CP.ok(x, w, b) and out_dtype == torch.float32:
        Nn, Cx, H, W = x.shape
        K, Cg, R, S = w.shape
        if Cx != Cg * groups or K % groups:
            raise ValueError(f"conv2d: input {tuple(x.shape)} / weight {tuple(w.shape)} / groups {groups} mismatch")
        Ho, Wo = conv_out_size(H, R, sh, ph, dh), conv_out_size(W, S, sw, pw, dw)
        xc, wc = CP.dense32(x), CP.dense32(w)
        y = _mem.empty((Nn, K, Ho, Wo), dtype=torch.float32)
        CP.lib().conv_fwd(xc.data_ptr(), wc.data_ptr(), CP.p(CP.dense32(b) if b is not None else None), y.data_ptr(),
                          Nn, Cx, H, W, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, groups)
        return unary("relu", y) if relu else y
    xf = x.float() if x.dtype != torch.float32 else x
    y = F.conv2d(xf, w.float(), b.float() if b is not None else None, (sh, sw), (ph, pw), (dh, dw), groups)
    if relu:
        y = torch.relu(y)
    return y.to(out_dtype)


# conv data gradient reads the weights K-major from a per-call transposed copy
# (ds_read_b128 fragments like the forward) instead of transposing them
# through LDS (ds_read_b64_tr_b16); switchable for A/B measurements
DGRAD_KMAJOR = os.environ.get("SINGA_AMD_DGRAD_KMAJOR", "1") != "0"
# a conv dgrad whose input came from a BN+ReLU can sum that BN backward's
# partials in its epilogue.  Off by default since the separate reduction
# streams at 6+ TB/s (contiguous spans, non-temporal loads): ResNet-50 b1024
# 12.22k img/s unfused vs 11.81k fused (A/B in one session on MI355X)
FUSE_BN_BWD_STATS = os.environ.get("SINGA_AMD_FUSE_BN_BWD", "0") == "1"
# residual BN(+ReLU) backward partials in the completing dgrad's epilogue:
# measured break-even on MI355X (tools/bench_dgrad_bn.py: the extra BN-input
# read in the epilogue of these one/two-K-tile GEMMs costs what the separate
# reduction pass costs, profiles/dgrad_bn_fusion_b1024.jsonl), so off by default
FUSE_RES_BN_BWD = os.environ.get("SINGA_AMD_FUSE_RES_BN_BWD", "0") == "1"
# Identity-sum BN backward (bn_bwd_finalize_wdot_k, batchnorm.hip): a
# BN(+ReLU) whose output feeds exactly one conv skips its reduction pass;
# sum(g~) comes from that conv's dgrad epilogue (mask bits) and sum(g~ xhat)
# from <W, dW> of its weight gradient
BN_WDOT_MODE = int(os.environ.get("SINGA_AMD_BN_WDOT", "1"))  # 0 off, 1 every consuming conv, 2 only 1x1 ones
BN_WDOT = BN_WDOT_MODE > 0
BN_WDOT_TAU = 0.05  # |gamma| below this (or |beta| > 4 |gamma|): the exact reduction runs instead


_WT_CACHE: dict = {}
# set to a list by Model._run_graph while it captures a HIP graph: every cached
# scratch / descriptor entry a captured launch addresses is appended, and the
# graph keeps the list alive (an evicted entry then lives exactly as long as
# the graphs that replay into it)
CAPTURE_KEEP: Optional[list] = None


def pretranspose_conv_weights(items) -> dict:
    """K-major copies ([R*S][C][K]) of every conv weight a backward pass will
    need for its data gradients, written by ONE batched launch instead of one
    small transpose launch in front of each dgrad.  ``items``: (key, w) with w
    the bf16 channels-last weight the forward used.  Returns {key: wt}.  The
    descriptor table and scratch are cached per weight set (stable pointers
    in the flat parameter store), so a captured step replays just the launch."""
    sel = []
    for key, w in items:
        if (w is not None and w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 4 and N.is_cl(w)
                and w.shape[0] % 64 == 0 and w.shape[1] % 8 == 0):
            sel.append((key, w))
    if len(sel) < 2 or not DGRAD_KMAJOR:
        return {}
    # one scratch per (weight set, thread): replica threads sharing the
    # weights run on their own streams and must not write each other's copy.
    # Keyed by thread, not stream: a HIP-graph capture runs the same step on a
    # side stream and must hit the entry its eager warm-up created
    sig = tuple((w.data_ptr(),) + tuple(w.shape) for _, w in sel) + (threading.get_ident(),)
    ent = _WT_CACHE.get(sig)
    if ent is None:
        if len(_WT_CACHE) > 8:
            # evict: a captured HIP graph that replays into an entry holds it
            # through its CAPTURE_KEEP list, so dropping the cache's
            # reference here frees only entries no live graph addresses
            _WT_CACHE.clear()
        dev = sel[0][1].device
        sizes = [w.numel() for _, w in sel]
        offs = np.cumsum([0] + [(n + 63) // 64 * 64 for n in sizes])
        scratch = _mem.empty(int(offs[-1]), dtype=torch.bfloat16, device=dev)
        desc = np.zeros((len(sel), 4), dtype=np.int64)
        tile0 = 0
        for i, (_, w) in enumerate(sel):
            K, C, R, S = w.shape
            desc[i, 0] = w.data_ptr()
            desc[i, 1] = scratch.data_ptr() + 2 * int(offs[i])
            desc[i, 2] = K | ((R * S) << 32)
            desc[i, 3] = C | (tile0 << 32)
            tile0 += ((C + 63) // 64) * ((K + 63) // 64) * R * S
        # pinned source: a copy issued while a step is being captured becomes a
        # graph node (a pageable one is not permitted); kept alive in the entry
        host = torch.from_numpy(desc).pin_memory()
        ent = (host.to(dev, non_blocking=True), scratch, [scratch[int(o):int(o) + n] for o, n in zip(offs, sizes)],
               tile0, host)
        _WT_CACHE[sig] = ent
    if CAPTURE_KEEP is not None:
        CAPTURE_KEEP.append(ent)
    desc_dev, _, views, total, _ = ent
    N.lib().wt_transpose_batched(desc_dev.data_ptr(), len(sel), total, N.stream())
    return {key: v for (key, _), v in zip(sel, views)}


def _conv_bwd_res(x, w, dy, stride, padding, dw_out, need_db, mg: "MaskedGrad", wt_pre, db_out):
    """conv2d_bwd with a lazy residual gradient to absorb: dx = dgrad +
    g * bit(mask) in the dgrad epilogue (native bf16, stride 1); the weight
    / bias gradients as in conv2d_bwd."""
    Nn, C, H, W = x.shape
    K, _, R, S = w.shape
    Ho, Wo = dy.shape[2], dy.shape[3]
    dyb = dy if (dy.dtype == torch.bfloat16 and N.is_cl(dy)) else to_nhwc_bf16(dy, K)
    wb = w if (w.dtype == torch.bfloat16 and N.is_cl(w)) else G.to(w, torch.bfloat16, torch.channels_last)
    wt, ready = None, False
    if DGRAD_KMAJOR and K % 64 == 0:
        if wt_pre is not None and wb is w and wt_pre.numel() == K * C * R * S:
            wt, ready = wt_pre, True
        else:
            wt = _mem.empty(K * C * R * S, dtype=torch.bfloat16, device=x.device)
    if ready:
        N.lib().set_wt_ready(1)
    dxp = _mem.empty((Nn, C, H, W), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    g = mg.g if N.is_cl(mg.g) else G.contiguous(mg.g, torch.channels_last)
    ok = N.lib().conv_dgrad_res(dyb.data_ptr(), wb.data_ptr(), dxp.data_ptr(), Nn, H, W, C, K, R, S, Ho, Wo,
                                stride[0], stride[1], padding[0], padding[1], 1, 1, N.ptr(wt), g.data_ptr(),
                                mg.mask.data_ptr(), N.stream())
    if not ok:  # shape the epilogue cannot take: materialise and accumulate as usual
        return conv2d_bwd(x, w, dy, stride, padding, (1, 1), 1, True, dw_out, need_db, mg.materialize(), None,
                          None, db_out)
    mg.value = dxp
    mg.g = mg.mask = None
    dxp._sg_fresh = True
    # weight (and bias) gradient: the plain path with no data gradient
    _, dwt, db = conv2d_bwd(x, w, dy, stride, padding, (1, 1), 1, False, dw_out, need_db, None, None, None, db_out)
    return mg, dwt, db


def conv2d_bwd(x: torch.Tensor, w: torch.Tensor, dy: torch.Tensor, stride, padding, dilation=(1, 1), groups=1,
               need_dx=True, dw_out: Optional[torch.Tensor] = None, need_db=False,
               dx_acc: Optional[torch.Tensor] = None, bn_producer=None, wt_pre: Optional[torch.Tensor] = None,
               db_out: Optional[torch.Tensor] = None, bn_wdot: bool = False):
    """Returns (dx, dw, db).  If dw_out (fp32, same logical shape as w) is given
    the weight gradient is ACCUMULATED into it (flat grad buffer views); the
    same for the bias gradient with ``db_out`` (fp32 [K]).
    ``dx_acc``: an existing gradient of x (another consumer's contribution);
    when its layout allows, the data gradient is added into it in the dgrad
    epilogue and ``dx_acc`` itself is returned as dx.
    ``bn_producer`` = (x_bn, BNState): x is the output of a training-mode
    BatchNorm+ReLU (no residual) whose pre-BN input is x_bn; the dgrad
    epilogue then also sums that BN backward's per-channel partials and
    attaches them to dx (``dx._sg_bnbwd_ws``) so its reduction pass is skipped.
    ``bn_producer`` = (x_bn, BNState, mask) with ``dx_acc``: the producer is a
    residual BN(+ReLU) with a 1-bit ReLU mask and this accumulation is the
    last contribution to its output gradient: same fusion, on ``dx_acc``."""
    sh, sw = stride
    ph, pw = padding
    dh, dw_ = dilation
    strided = None
    if isinstance(dx_acc, StridedGrad):
        # kept compact only into a gmask (fused-tail) dgrad of a 1x1 / stride-1 conv
        if (need_dx and dx_acc.value is None and bn_producer is not None and isinstance(bn_producer[0], str)
                and bn_producer[0] == "gmask" and _native_ok(x, w, dy) and groups == 1
                and x.dtype == torch.bfloat16 and tuple(w.shape[2:]) == (1, 1) and sh == sw == 1 and ph == pw == 0
                and dh == dw_ == 1 and tuple(dx_acc.shape) == tuple(x.shape) and dx_acc.dtype == torch.bfloat16
                and x.shape[1] % 8 == 0 and not N.lib().deterministic()):
            strided = dx_acc
        else:
            dx_acc = dx_acc.materialize()
    if isinstance(dx_acc, MaskedGrad):
        K_, C_ = w.shape[0], w.shape[1]
        if (need_dx and _native_ok(x, w, dy) and groups == 1 and x.dtype == torch.bfloat16 and C_ % 8 == 0
                and K_ % 8 == 0 and x.shape[1] == C_ and tuple(dx_acc.shape) == tuple(x.shape)
                and dx_acc.dtype == torch.bfloat16 and dx_acc.value is None and sh == 1 and sw == 1
                and dh == 1 and dw_ == 1 and not N.lib().deterministic()):
            return _conv_bwd_res(x, w, dy, stride, padding, dw_out, need_db, dx_acc, wt_pre, db_out)
        dx_acc = dx_acc.materialize()
    if _native_ok(x, w, dy) and not (groups == 1 and x.dtype == torch.bfloat16 and
                                     (not need_dx or (dh == 1 and dw_ == 1 and sh * sw <= 16))):
        return _gconv_bwd(x, w, dy, stride, padding, dilation, groups, need_dx, dw_out, need_db, dx_acc, db_out)
    if _native_ok(x, w, dy) and groups == 1:
        Nn, Cx, H, W = x.shape
        K, C, R, S = w.shape
        Ho, Wo = dy.shape[2], dy.shape[3]
        Cp, Kp = _pad8(C), _pad8(K)
        xb = x if (x.dtype == torch.bfloat16 and N.is_cl(x) and Cx == Cp) else to_nhwc_bf16(x[:, :C], Cp)
        dyb = dy if (dy.dtype == torch.bfloat16 and N.is_cl(dy) and Kp == K) else to_nhwc_bf16(dy, Kp)
        padded = Cp != C or Kp != K
        dx = dwt = db = None
        if need_dx:
            if dh != 1 or dw_ != 1:
                raise NotImplementedError("GPU conv data-gradient with dilation > 1")
            if sh * sw > 16:
                raise NotImplementedError("GPU conv data-gradient with stride_h*stride_w > 16")
            if padded:
                wb = _zeros_cl((Kp, Cp, R, S), torch.bfloat16, w.device)
                G.copy_(wb[:K, :C], w)
            else:
                wb = w if (w.dtype == torch.bfloat16 and N.is_cl(w)) else G.to(w, torch.bfloat16,
                                                                                 torch.channels_last)
            od = torch.bfloat16 if x.dtype == torch.bfloat16 else torch.float32
            om = 0 if od == torch.bfloat16 else 1
            # K-major transposed weights for the B operand: the batched pre-pass's
            # copy (``wt_pre``) or scratch the dgrad call transposes into
            wt, ready = None, False
            if DGRAD_KMAJOR and Kp % 64 == 0:
                if wt_pre is not None and not padded and wb is w and wt_pre.numel() == Kp * Cp * R * S:
                    wt, ready = wt_pre, True
                else:
                    wt = _mem.empty(Kp * Cp * R * S, dtype=torch.bfloat16, device=x.device)
            if ready:
                N.lib().set_wt_ready(1)  # one-shot: consumed by the dgrad launch below
            gmask = (bn_producer[1] if bn_producer is not None and isinstance(bn_producer[0], str)
                     and bn_producer[0] == "gmask" else None)
            if gmask is not None:
                bn_producer = None
                if not (od == torch.bfloat16 and Cx == Cp and C % 8 == 0 and not padded
                        and not N.lib().deterministic()
                        and (dx_acc is None or strided is not None
                             or (dx_acc.dtype == od and tuple(dx_acc.shape) == tuple(x.shape) and N.is_cl(dx_acc)
                                 and dx_acc.is_contiguous(memory_format=torch.channels_last)))):
                    gmask = None  # (the consumer then masks and sums the gradient itself)
                    if strided is not None:
                        dx_acc, strided = strided.materialize(), None
            if gmask is not None:
                # the consumer is a fused residual tail (ConvBNAddReLU): this dgrad
                # completes its output gradient, so the epilogue writes it masked
                # (g = d(out) * bit) and sums it per channel (stats_mode 4)
                # (the other consumers' gradient dx_acc is added from its own
                # buffer into a fresh dx, beta = 0: the single-stage short-K
                # variant stays available; the caller replaces dx_acc by it)
                dxp = _mem.empty((Nn, Cp, H, W), dtype=od, device=x.device, memory_format=torch.channels_last)
                bws = zeroed_ws(32 * 2 * C, x.device)
                acc_t, acc_s = (strided.g, strided.stride) if strided is not None else (dx_acc, 1)
                N.lib().conv_dgrad_gsum(dyb.data_ptr(), wb.data_ptr(), dxp.data_ptr(), Nn, H, W, Cp, Kp, R, S, Ho,
                                        Wo, sh, sw, ph, pw, dh, dw_, N.ptr(wt), N.ptr(acc_t), bws.data_ptr(),
                                        gmask.data_ptr(), acc_s, acc_t.shape[2] if acc_t is not None else 0,
                                        acc_t.shape[3] if acc_t is not None else 0, N.stream())
                dxp._sg_gsum = (bws, gmask)
                dxp._sg_fresh = True
                if dx_acc is not None:
                    dxp._sg_absorbed = dx_acc
                dx = dxp
            elif (dx_acc is not None and Cx == Cp and dx_acc.dtype == od and od == x.dtype
                    and tuple(dx_acc.shape) == tuple(x.shape) and N.is_cl(dx_acc) and dx_acc.is_contiguous(
                        memory_format=torch.channels_last)):
                bmask = bn_producer[2] if bn_producer is not None and len(bn_producer) > 2 else None
                if (bmask is not None and FUSE_BN_BWD_STATS and FUSE_RES_BN_BWD and od == torch.bfloat16 and C % 8 == 0
                        and not N.lib().deterministic() and bn_producer[0].dtype == torch.bfloat16
                        and tuple(bn_producer[0].shape) == tuple(x.shape) and N.is_cl(bn_producer[0])
                        and bn_producer[0].is_contiguous(memory_format=torch.channels_last)):
                    # this accumulation completes the gradient of a residual
                    # BN(+ReLU) output: the epilogue also sums that BN
                    # backward's partials from the final values (its 1-bit
                    # ReLU mask), so the BN skips its reduction pass
                    xbn, bst = bn_producer[0], bn_producer[1]
                    bws = zeroed_ws(32 * 2 * C, x.device)
                    N.lib().conv_dgrad_bn(dyb.data_ptr(), wb.data_ptr(), dx_acc.data_ptr(), Nn, H, W, Cp, Kp, R, S, Ho,
                                          Wo, sh, sw, ph, pw, dh, dw_, N.ptr(wt), bws.data_ptr(), xbn.data_ptr(),
                                          bst.mean.data_ptr(), bst.invstd.data_ptr(), bst.scale.data_ptr(),
                                          bst.shift.data_ptr(), N.stream(), 1.0, bmask.data_ptr())
                    dx_acc._sg_bnbwd_ws = (bws, 32)
                else:
                    N.lib().conv_dgrad_acc(dyb.data_ptr(), wb.data_ptr(), dx_acc.data_ptr(), Nn, H, W, Cp, Kp, R, S,
                                           Ho, Wo, sh, sw, ph, pw, dh, dw_, om, 1.0, N.stream(), N.ptr(wt))
                dx = dx_acc
            elif (bn_wdot and bn_producer is not None and od == torch.bfloat16 and Cx == Cp and C % 8 == 0
                  and not padded and not N.lib().deterministic() and x.dtype == torch.bfloat16):
                # identity-sum BN backward of the producer BN(+ReLU): this
                # dgrad's epilogue sums the masked gradient (mask bits only)
                bmask = bn_producer[2]
                dxp = _mem.empty((Nn, Cp, H, W), dtype=od, device=x.device, memory_format=torch.channels_last)
                bws = zeroed_ws(32 * 2 * C, x.device)
                N.lib().conv_dgrad_bn(dyb.data_ptr(), wb.data_ptr(), dxp.data_ptr(), Nn, H, W, Cp, Kp, R, S, Ho, Wo,
                                      sh, sw, ph, pw, dh, dw_, N.ptr(wt), bws.data_ptr(), 0, 0, 0, 0, 0, N.stream(),
                                      0.0, bmask.data_ptr())
                dxp._sg_bnbwd_wdot = (bws, None, wb, bn_producer[3], bn_producer[4])  # (.., gamma, beta)
                dxp._sg_fresh = True
                dx = dxp
            elif (bn_producer is not None and FUSE_BN_BWD_STATS and od == torch.bfloat16 and Cx == Cp and C % 8 == 0
                  and not N.lib().deterministic() and bn_producer[0].dtype == torch.bfloat16
                  and tuple(bn_producer[0].shape) == tuple(x.shape) and N.is_cl(bn_producer[0])
                  and bn_producer[0].is_contiguous(memory_format=torch.channels_last)):
                xbn, bst = bn_producer
                dxp = _mem.empty((Nn, Cp, H, W), dtype=od, device=x.device, memory_format=torch.channels_last)
                bws = zeroed_ws(32 * 2 * C, x.device)
                N.lib().conv_dgrad_bn(dyb.data_ptr(), wb.data_ptr(), dxp.data_ptr(), Nn, H, W, Cp, Kp, R, S, Ho, Wo,
                                      sh, sw, ph, pw, dh, dw_, N.ptr(wt), bws.data_ptr(), xbn.data_ptr(),
                                      bst.mean.data_ptr(), bst.invstd.data_ptr(), bst.scale.data_ptr(),
                                      bst.shift.data_ptr(), N.stream())
                dxp._sg_bnbwd_ws = (bws, 32)
                dxp._sg_fresh = True
                dx = dxp
            else:
                dxp = _mem.empty((Nn, Cp, H, W), dtype=od, device=x.device, memory_format=torch.channels_last)
                N.lib().conv_dgrad_acc(dyb.data_ptr(), wb.data_ptr(), dxp.data_ptr(), Nn, H, W, Cp, Kp, R, S, Ho, Wo,
                                       sh, sw, ph, pw, dh, dw_, om, 0.0, N.stream(), N.ptr(wt))
                dx = G.contiguous(dxp[:, :C], torch.channels_last) if Cx != Cp else dxp
                if dx.dtype != x.dtype:
                    dx = cast(dx, x.dtype)
                dx._sg_fresh = True
        # weight gradient, fp32 [Kp][R][S][Cp]
        direct = (dw_out is not None and not padded and dw_out.dtype == torch.float32 and N.is_cl(dw_out))
        target = dw_out if direct else _zeros_cl((Kp, Cp, R, S), torch.float32, x.device)
        N.lib().conv_wgrad(xb.data_ptr(), dyb.data_ptr(), target.data_ptr(), Nn, H, W, Cp, Kp, R, S, Ho, Wo, sh, sw,
                           ph, pw, dh, dw_, 0, N.stream())
        wd = getattr(dx, "_sg_bnbwd_wdot", None) if dx is not None else None
        if wd is not None:
            # <W, dW> per input channel over the finished weight gradient (the
            # caller guarantees it held nothing else before this backward)
            wdot = zeroed_ws(C + 1, x.device)  # [C] sums + the producer BN's gate flag (int)
            N.lib().wdot_colsum(wd[2].data_ptr(), target.data_ptr(), Kp * R * S, C, 1.0, wdot.data_ptr(), 1,
                                wd[3].data_ptr(), wd[4].data_ptr(), BN_WDOT_TAU, N.stream())
            dx._sg_bnbwd_wdot = (wd[0], wdot)
        if direct:
            dwt = dw_out
        else:
            g = target[:K, :C]
            if dw_out is not None:
                dwt = G.binary("add", dw_out, g, out=dw_out)
            else:
                dwt = G.contiguous(g)
        if need_db:
            acc = Kp == K and _db_ok(db_out, K)
            db = colsum(dyb.permute(0, 2, 3, 1).reshape(-1, Kp), out=db_out.view(-1) if acc else None)[0][:K]
            if db_out is not None and not acc:
                db = G.binary("add", db_out, G.reshape(db, db_out.shape), out=db_out)
        return dx, dwt, db
    _no_native("conv2d_bwd", x, w, dy)
    if CP.ok(x, w, dy):
        Nn, Cx, H, W = x.shape
        K, Cg, R, S = w.shape
        Ho, Wo = dy.shape[2], dy.shape[3]
        xc, wc, dyc = CP.dense32(x), CP.dense32(w), CP.dense32(dy)
        dx = _mem.empty(x.shape, dtype=torch.float32) if need_dx else None
        direct = dw_out is not None and CP.ok(dw_out) and dw_out.is_contiguous()
        dwt = dw_out if direct else G.zeros(tuple(w.shape), torch.float32, x.device)
        db = None
        if need_db:
            db = db_out if _db_ok(db_out, K) else G.zeros((K,), torch.float32, x.device)
        CP.lib().conv_bwd(xc.data_ptr(), wc.data_ptr(), dyc.data_ptr(), CP.p(dx), dwt.data_ptr(), CP.p(db), Nn, Cx, H,
                          W, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw_, groups)
        if dw_out is not None and not direct:
            dwt = G.binary("add", dw_out, dwt, out=dw_out)
        if db is not None and db_out is not None and db is not db_out:
            db = G.binary("add", db_out, G.reshape(db, db_out.shape), out=db_out)
        return dx, dwt, db
    # CPU reference via autograd of the functional conv
    with torch.enable_grad():
        xx = x.detach().float().requires_grad_(need_dx)
        ww = w.detach().float().requires_grad_(True)
        y = F.conv2d(xx, ww, None, (sh, sw), (ph, pw), (dh, dw_), groups)
        grads = torch.autograd.grad(y, [xx, ww] if need_dx else [ww], dy.float())
    dx = grads[0].to(x.dtype) if need_dx else None
    gw = grads[-1]
    if dw_out is not None:
        dw_out.add_(gw)
        gw = dw_out
    db = dy.float().sum(dim=(0, 2, 3)) if need_db else None
    if db is not None and db_out is not None:
        db = db_out.add_(db.reshape(db_out.shape))
    return dx, gw, db


# ----------------------------------------------------------------------------
# reductions, batchnorm, pooling, LRN
# ----------------------------------------------------------------------------
def _rows_c(x: torch.Tensor) -> Tuple[torch.Tensor, int, int]:
    """View a channels_last 4-D (or 2-D [R,C]) tensor as [R][C] memory."""
    if x.dim() == 4:
        if not N.is_cl(x):
            raise ValueError("expected channels_last tensor")
        C = x.shape[1]
        return x, x.numel() // C, C
    return x, x.shape[0], x.shape[-1]


_BANDS: dict = {}


class _ZeroArena:
    """Per-training-step arena of ZEROED fp32 scratch for the slot-atomic
    reduction workspaces (BatchNorm statistics / backward partial sums and
    the conv-epilogue BN statistics).  ``begin()`` zeroes the whole arena with
    ONE kernel at the start of a step; a launch whose workspace comes from the
    arena tells the kernel library it is pre-zeroed (a host flag read at
    launch time), which replaces ~2 zeroing launches per BatchNorm layer
    (~100 per ResNet-50 step).  Sizes settle after the first step (high-water
    mark), so a HIP-graph capture never reallocates."""

    def __init__(self):
        self.buf: Optional[torch.Tensor] = None
        self.retired: list = []
        self.off = 0
        self.hwm = 0
        self.active = False
        self.hits = self.misses = 0  # of the current / last step

    def begin(self, device) -> None:
        if not N.available() or device.type != "cuda" or N.lib().deterministic():
            return
        if self.hwm > 0 and (self.buf is None or self.buf.numel() < self.hwm or self.buf.device != device):
            if self.buf is not None:  # a captured HIP graph may still address it: never free
                self.retired.append(self.buf)
            self.buf = _mem.empty(self.hwm + self.hwm // 8 + 1024, dtype=torch.float32, device=device)
        self.off = 0
        self.active = True
        self.hits = self.misses = 0
        if self.buf is not None:
            N.lib().zero(self.buf.data_ptr(), self.buf.numel() * 4, N.stream())

    def take(self, n: int, device) -> Optional[torch.Tensor]:
        """A zeroed slice of n floats, or None (arena inactive / too small)."""
        if not self.active:
            return None
        n = (n + 63) // 64 * 64
        end = self.off + n
        self.off = end  # advances on a miss too: the next begin() sizes for the whole step
        self.hwm = max(self.hwm, end)
        if self.buf is None or end > self.buf.numel() or self.buf.device != device:
            self.misses += 1
            return None
        t = self.buf[end - n:end]
        self.hits += 1
        return t

    def end(self) -> None:
        self.active = False


class _ThreadArenas(threading.local):
    """One arena per OS thread: replica threads (hogwild / aggregated
    executors, the loopback communicator's ranks) run their steps
    concurrently on their own streams, and the C++ 'pre-zeroed' flag the arena
    drives is per thread as well."""

    def __init__(self):
        self.arena = _ZeroArena()


_ARENAS = _ThreadArenas()


class _ArenaProxy:
    def __getattr__(self, k):
        return getattr(_ARENAS.arena, k)


ARENA = _ArenaProxy()


def zeroed_ws(n: int, device) -> torch.Tensor:
    """fp32 slot-atomic workspace of n floats for the NEXT native launch:
    an arena slice (pre-zeroed: the kernel skips its zeroing) or a fresh
    buffer (the kernel zeroes it)."""
    t = ARENA.take(n, device)
    if N.available():
        N.lib().set_ws_prezeroed(1 if t is not None else 0)
    return t if t is not None else _mem.empty(n, dtype=torch.float32, device=device)


def _ws(R: int, C: int, device) -> torch.Tensor:
    """Partial-sum workspace of a [R][C] column reduction."""
    key = (R, C, N.lib().deterministic())
    n = _BANDS.get(key)
    if n is None:
        n = _BANDS[key] = N.lib().colreduce_ws(R, C)
    return zeroed_ws(n, device)


def colsum(x2: torch.Tensor, with_sq: bool = False, out: Optional[torch.Tensor] = None):
    """Per-column sum (and sum of squares) of a [R, C] row-major tensor -> fp32.
    If ``out`` is given the column sums are ACCUMULATED into it."""
    if _native_ok(x2) and x2.dtype in (torch.float32, torch.bfloat16):
        x2 = G.contiguous(x2)
        R, C = x2.shape
        o0 = out if out is not None else _mem.empty(C, dtype=torch.float32, device=x2.device)
        o1 = _mem.empty(C, dtype=torch.float32, device=x2.device) if with_sq else None
        N.lib().colsum(x2.data_ptr(), _ws(R, C, x2.device).data_ptr(), o0.data_ptr(), N.ptr(o1), R, C, N.dt(x2),
                       int(out is not None), N.stream())
        return o0, o1
    _no_native("colsum", x2)
    if CP.ok(x2, out):
        s0 = G.reduce(x2, [0], "sum")
        if out is not None:
            s0 = G.binary("add", out, s0, out=out)
        return s0, (G.reduce(x2, [0], "sumsq") if with_sq else None)
    xf = x2.float()
    s0 = xf.sum(0)
    if out is not None:
        out.add_(s0)
        s0 = out
    return s0, ((xf * xf).sum(0) if with_sq else None)


class BNState:
    """Saved tensors of a batch-norm forward needed by the backward.
    ``mask``: 1-bit ReLU mask [R][C/8] of a fused BN(+residual)+ReLU output
    (written by the forward apply when requested; the backward then reads it
    instead of the bf16 output)."""
    __slots__ = ("mean", "invstd", "scale", "shift", "mask", "colsum")

    def __init__(self, mean, invstd, scale, shift, mask=None):
        self.mean, self.invstd, self.scale, self.shift, self.mask = mean, invstd, scale, shift, mask
        self.colsum = None  # column sums of the output (want_colsum)


# lazy residual gradient (see MaskedGrad); SINGA_AMD_LAZY_RES=0 writes it as a tensor
LAZY_RES = os.environ.get("SINGA_AMD_LAZY_RES", "1") != "0"


class MaskedGrad:
    """The gradient a residual BN(+ReLU) passes to its shortcut input, kept
    LAZY as (g, 1-bit ReLU mask): g * bit(mask).  The autograd engine holds it
    like a partial gradient; a conv whose data gradient completes that input
    adds it in its dgrad epilogue straight from (g, mask) (conv_dgrad_res),
    so the BN backward never writes it and nobody reads it back as a bf16
    tensor.  Any other consumer gets :meth:`materialize` (one native masking
    pass).  ``value``: set once absorbed or materialised."""

    _sg_fresh = True  # the engine owns it exclusively (may be absorbed in place)

    def __init__(self, g: torch.Tensor, mask: torch.Tensor):
        self.g, self.mask, self.value = g, mask, None
        self.shape, self.dtype, self.device = g.shape, g.dtype, g.device

    def is_floating_point(self) -> bool:
        return True

    def materialize(self) -> torch.Tensor:
        if self.value is None:
            out = _like(self.g)
            N.lib().mask_bits_apply(self.g.data_ptr(), self.mask.data_ptr(), out.data_ptr(), self.g.numel(),
                                    N.stream())
            out._sg_fresh = True
            self.value = out
            self.g = self.mask = None
        return self.value


class StridedGrad:
    """The input gradient of a strided 1x1 shortcut conv kept COMPACT: g is
    [N, C, H/s, W/s] (every s-th pixel of the input grid; zero elsewhere).  A
    consuming 1x1 conv's data gradient adds it in its epilogue straight from
    the compact tensor (conv_dgrad_gsum with acc_s = s), so the full-grid
    tensor -- three quarters zeros -- is never written nor read back.  Any
    other consumer gets :meth:`materialize` (strided_place)."""

    _sg_fresh = True  # the engine owns it exclusively

    def __init__(self, g: torch.Tensor, stride: int, shape):
        self.g, self.stride, self.value = g, int(stride), None
        self.shape, self.dtype, self.device = torch.Size(shape), g.dtype, g.device

    def is_floating_point(self) -> bool:
        return True

    def materialize(self) -> torch.Tensor:
        if self.value is None:
            self.value = strided_place(self.g, tuple(self.shape), self.stride)
            self.g = None
        return self.value


STRIDED_LAZY = os.environ.get("SINGA_AMD_STRIDED_LAZY", "1") != "0"  # (A/B: place the shortcut gradient eagerly)
LAZY_GRADS = (MaskedGrad, StridedGrad)  # gradient placeholders the autograd engine materialises on demand


def _bn_native(x: torch.Tensor) -> bool:
    return _native_ok(x) and _flat_ok(x) and ((x.dim() == 2 and x.is_contiguous()) or N.is_cl(x))


def _bn_params(x: torch.Tensor, gamma, beta, run_mean, run_var, training: bool, momentum: float, eps: float):
    """Native path: (mean, invstd, scale, shift) of a BN over x (training:
    batch statistics -- from the producing conv's epilogue sums when present
    -- and a running-stat update; inference: running statistics)."""
    L = N.lib()
    C = x.shape[1]
    R = x.numel() // C
    dev = x.device
    p = _mem.empty(4 * C, dtype=torch.float32, device=dev)
    mean, invstd, scale, shift = p[:C], p[C:2 * C], p[2 * C:3 * C], p[3 * C:]
    pre = getattr(x, "_sg_bn_ws", None)  # statistics already summed by the producing conv's epilogue
    if training and pre is not None and pre[0].numel() == pre[1] * 2 * C:
        L.bn_fwd_from_ws(pre[0].data_ptr(), pre[1], gamma.data_ptr(), beta.data_ptr(), run_mean.data_ptr(),
                         run_var.data_ptr(), mean.data_ptr(), invstd.data_ptr(), scale.data_ptr(),
                         shift.data_ptr(), R, C, momentum, eps, N.stream())
    elif training:
        L.bn_fwd_stats(x.data_ptr(), _ws(R, C, dev).data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                       run_mean.data_ptr(), run_var.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                       scale.data_ptr(), shift.data_ptr(), R, C, momentum, eps, N.dt(x), N.stream())
    else:
        L.bn_infer_params(gamma.data_ptr(), beta.data_ptr(), run_mean.data_ptr(), run_var.data_ptr(),
                          scale.data_ptr(), shift.data_ptr(), mean.data_ptr(), invstd.data_ptr(), C, eps,
                          N.stream())
    return mean, invstd, scale, shift


def bn_relu_maxpool_ok(x: torch.Tensor, kernel, stride, padding, ceil_mode: bool = False) -> bool:
    """The fused BN+ReLU+max-pool kernel applies (bf16 NHWC, C % 8 == 0, windows < 256 taps)."""
    return (_bn_native(x) and x.dim() == 4 and x.dtype == torch.bfloat16 and N.is_cl(x) and x.shape[1] % 8 == 0
            and not ceil_mode and kernel[0] * kernel[1] < 256)


def bn_relu_maxpool_fwd(x: torch.Tensor, gamma, beta, run_mean, run_var, training: bool, momentum: float,
                        eps: float, kernel, stride, padding):
    """max_pool(relu(BN(x))) in one pass over x (native, see bn_relu_maxpool_ok).
    Returns (y, arg, BNState): the BN output itself is never materialised;
    the backward is pool2d_bwd (argmax gather) then batchnorm_bwd with the
    ReLU mask recomputed from x."""
    mean, invstd, scale, shift = _bn_params(x, gamma, beta, run_mean, run_var, training, momentum, eps)
    kh, kw = kernel
    sh, sw = stride
    ph, pw = padding
    Nn, C, H, W = x.shape
    Ho = (H + 2 * ph - kh) // sh + 1
    Wo = (W + 2 * pw - kw) // sw + 1
    y = _mem.empty((Nn, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    arg = _mem.empty((Nn, Ho, Wo, C), dtype=torch.uint8, device=x.device)
    N.lib().bn_relu_maxpool(x.data_ptr(), scale.data_ptr(), shift.data_ptr(), y.data_ptr(), arg.data_ptr(), Nn, H, W,
                            C, Ho, Wo, kh, kw, sh, sw, ph, pw, N.stream())
    return y, arg, BNState(mean, invstd, scale, shift, None)


def _fuse_pool_bwd() -> bool:
    # opt-in: measured 12.98k vs 13.09k img/s (ResNet-50 b1024, A/B/A in one
    # session) -- the per-row argmax gather in BOTH BN passes costs more VALU
    # than the 1.6 GB write + two reads of the max-pool backward output save
    return os.environ.get("SINGA_AMD_FUSE_POOL_BWD", "0") == "1"


def bn_relu_maxpool_bwd(x: torch.Tensor, dy: torch.Tensor, arg: torch.Tensor, gamma: torch.Tensor, st: "BNState",
                        kernel, stride, padding, dg_out=None, db_out=None):
    """Backward of :func:`bn_relu_maxpool_fwd`: (dx, dgamma, dbeta).  Native:
    the BN backward gathers its input gradient from the pooled gradient and
    the 8-bit argmax inside its reduction and apply passes (the full-size
    max-pool backward output is never written).  dgamma / dbeta accumulate
    into dg_out / db_out when given."""
    Nn, C, H, W = x.shape
    Ho, Wo = dy.shape[2], dy.shape[3]
    if (_fuse_pool_bwd() and _bn_native(x) and x.dtype == torch.bfloat16 and N.is_cl(x) and C % 8 == 0
            and dy.dtype == torch.bfloat16 and arg is not None and arg.dtype == torch.uint8):
        dyc = G.contiguous(dy, torch.channels_last)
        R = x.numel() // C
        dg = dg_out if dg_out is not None else G.zeros((C,), torch.float32, x.device)
        db = db_out if db_out is not None else G.zeros((C,), torch.float32, x.device)
        coef = _mem.empty(3 * C, dtype=torch.float32, device=x.device)
        dx = _like(x)
        N.lib().bn_bwd_pool(x.data_ptr(), dyc.data_ptr(), arg.data_ptr(), st.scale.data_ptr(), st.shift.data_ptr(),
                            st.mean.data_ptr(), st.invstd.data_ptr(), gamma.data_ptr(), _ws(R, C, x.device).data_ptr(),
                            coef.data_ptr(), dg.data_ptr(), db.data_ptr(), dx.data_ptr(), Nn, H, W, C, Ho, Wo,
                            kernel[0], kernel[1], stride[0], stride[1], padding[0], padding[1], N.stream())
        dx._sg_fresh = True
        return dx, dg, db
    dpre = pool2d_bwd(x.shape, x, dy, arg, kernel, stride, padding, True)
    dx, dg, db, _ = batchnorm_bwd(x, dpre, gamma, st, None, need_dres=False, relu=True, dg_out=dg_out, db_out=db_out)
    return dx, dg, db


def batchnorm_fwd(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, run_mean: torch.Tensor,
                  run_var: torch.Tensor, training: bool, momentum: float = 0.1, eps: float = 1e-5,
                  relu: bool = False, residual: Optional[torch.Tensor] = None, want_mask: bool = False,
                  want_colsum: bool = False):
    """y = act(BN(x) + residual).  4-D x (channels_last on GPU) or 2-D [B, C].
    momentum follows the PyTorch convention (weight of the new statistic).
    ``want_mask`` (with relu, native path, C % 8 == 0): also write the 1-bit
    ReLU mask into the returned state (``st.mask``) for the backward.
    ``want_colsum`` (native bf16, no residual, C % 64 == 0): also the column
    sums of y (``st.colsum``, fp32 [32][C] slot rows) -- for a consuming fused residual
    tail (bnres_bwd), summed in this pass instead of re-reading y."""
    C = x.shape[1]
    if _bn_native(x):
        L = N.lib()
        R = x.numel() // C
        dev = x.device
        mean, invstd, scale, shift = _bn_params(x, gamma, beta, run_mean, run_var, training, momentum, eps)
        res = None
        if residual is not None:
            res = residual
            if res.dtype != x.dtype or not _same_layout(res, x):
                res = G.to(res, x.dtype, torch.channels_last if x.dim() == 4 else torch.contiguous_format)
        y = _like(x)
        mask = None
        if want_mask and relu and C % 8 == 0:
            mask = _mem.empty(R * C // 8, dtype=torch.uint8, device=dev)
        if want_colsum and res is None and x.dtype == torch.bfloat16 and C % 64 == 0:
            cs = _zeros32(32 * C, dev)  # 32 slot rows (the consumer sums them)
            L.bn_apply_cs(x.data_ptr(), scale.data_ptr(), shift.data_ptr(), y.data_ptr(), N.ptr(mask), cs.data_ptr(),
                          R, C, int(relu), N.stream())
            st = BNState(mean, invstd, scale, shift, mask)
            st.colsum = cs
            y._sg_cs_slots = cs  # (the consuming tail's forward statistics read them too)
            return y, st
        L.bn_apply(x.data_ptr(), scale.data_ptr(), shift.data_ptr(), N.ptr(res), y.data_ptr(), R, C, int(relu),
                   N.dt(x), N.stream(), N.ptr(mask))
        return y, BNState(mean, invstd, scale, shift, mask)
    # CPU reference
    _no_native("batchnorm_fwd", x)
    if (CP.ok(x, gamma, beta, run_mean, run_var, residual) and run_mean.is_contiguous() and run_var.is_contiguous()
            and x.dim() in (2, 4)):
        xc = CP.dense32(x)
        Nn = x.shape[0]
        HW = x.numel() // (Nn * C) if Nn * C else 0
        y = _mem.empty(x.shape, dtype=torch.float32)
        mean = _mem.empty(C, dtype=torch.float32)
        invstd = _mem.empty(C, dtype=torch.float32)
        res = CP.dense32(residual) if residual is not None else None
        CP.lib().bn_fwd(xc.data_ptr(), CP.dense32(gamma).data_ptr(), CP.dense32(beta).data_ptr(),
                        run_mean.data_ptr(), run_var.data_ptr(), y.data_ptr(), mean.data_ptr(), invstd.data_ptr(), Nn,
                        C, HW, int(training), float(momentum), float(eps), int(relu), CP.p(res))
        scale = G.binary("mul", gamma, invstd)
        shift = G.binary("sub", beta, G.binary("mul", mean, scale))
        return y, BNState(mean, invstd, scale, shift)
    dims = (0,) if x.dim() == 2 else (0, 2, 3)
    shp = (1, C) if x.dim() == 2 else (1, C, 1, 1)
    xf = x.float()
    if training:
        mean = xf.mean(dims)
        var = xf.var(dims, unbiased=False)
        cnt = x.numel() // C
        with torch.no_grad():
            run_mean.mul_(1 - momentum).add_(momentum * mean)
            run_var.mul_(1 - momentum).add_(momentum * var * cnt / max(cnt - 1, 1))
    else:
        mean, var = run_mean, run_var
    invstd = torch.rsqrt(var + eps)
    scale = gamma.float() * invstd
    shift = beta.float() - mean * scale
    y = xf * scale.reshape(shp) + shift.reshape(shp)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype), BNState(mean, invstd, scale, shift)


def dual_bn_add_relu_ok(x: torch.Tensor, x2: torch.Tensor) -> bool:
    """relu(BN(x) + BN2(x2)) runs fused: native, C % 8 == 0, same shape/layout."""
    return (_bn_native(x) and _bn_native(x2) and x.shape == x2.shape and x.dtype == x2.dtype
            and _same_layout(x, x2) and x.shape[1] % 8 == 0)


def dual_bn_add_relu_fwd(x, gamma, beta, rm, rv, x2, gamma2, beta2, rm2, rv2, training: bool, momentum: float,
                         eps: float, momentum2: float, eps2: float):
    """y = relu(BN(x) + BN2(x2)) in one pass (a residual block whose shortcut
    is a downsample conv + BN): BN2's output is never materialised.  Returns
    (y, st, st2); st.mask holds the 1-bit ReLU mask for the backward."""
    st_p = _bn_params(x, gamma, beta, rm, rv, training, momentum, eps)
    st2_p = _bn_params(x2, gamma2, beta2, rm2, rv2, training, momentum2, eps2)
    C = x.shape[1]
    R = x.numel() // C
    y = _like(x)
    mask = _mem.empty(R * C // 8, dtype=torch.uint8, device=x.device)
    N.lib().bn_apply2(x.data_ptr(), st_p[2].data_ptr(), st_p[3].data_ptr(), x2.data_ptr(), st2_p[2].data_ptr(),
                      st2_p[3].data_ptr(), y.data_ptr(), mask.data_ptr(), R, C, 1, N.dt(x), N.stream())
    return y, BNState(*st_p, mask), BNState(*st2_p, None)


def dual_bn_add_relu_bwd(x, dy, gamma, st: BNState, x2, gamma2, st2: BNState, dg_out=None, db_out=None,
                         dg2_out=None, db2_out=None):
    """Backward of dual_bn_add_relu_fwd: one reduction pass for both BNs, one
    apply pass writing dx and dx2.  Returns dx, dg, db, dx2, dg2, db2 (the
    parameter gradients accumulated into the *_out buffers when given)."""
    C = x.shape[1]
    R = x.numel() // C
    dev = x.device
    if dy.dtype != x.dtype or not _same_layout(dy, x):
        dy = G.to(dy, x.dtype, torch.channels_last if x.dim() == 4 else torch.contiguous_format)
    z = lambda o: o if o is not None else G.zeros((C,), torch.float32, dev)  # noqa: E731
    dg, db, dg2, db2 = z(dg_out), z(db_out), z(dg2_out), z(db2_out)
    key = (R, C, N.lib().deterministic())
    n = _BANDS.get(key)
    if n is None:
        n = _BANDS[key] = N.lib().colreduce_ws(R, C)
    wsb = zeroed_ws(2 * n, dev)  # one pre-zeroed flag for both halves (the kernel zeroes the second itself)
    coef = _mem.empty(6 * C, dtype=torch.float32, device=dev)
    dx, dx2 = _like(x), _like(x2)
    N.lib().bn_bwd2(x.data_ptr(), dy.data_ptr(), st.mask.data_ptr(), st.mean.data_ptr(), st.invstd.data_ptr(),
                    gamma.data_ptr(), x2.data_ptr(), st2.mean.data_ptr(), st2.invstd.data_ptr(), gamma2.data_ptr(),
                    wsb.data_ptr(), wsb[n:].data_ptr(), coef.data_ptr(), coef[3 * C:].data_ptr(), dg.data_ptr(),
                    db.data_ptr(), dg2.data_ptr(), db2.data_ptr(), dx.data_ptr(), dx2.data_ptr(), R, C, N.dt(x),
                    N.stream())
    dx._sg_fresh = True
    dx2._sg_fresh = True
    return dx, dg, db, dx2, dg2, db2


# ---------------------------------------------------------------------------
# Algebraic residual-tail backward (csrc/kernels/bnres.hip): out = relu(BN(W y)
# + res) for a 1x1 conv W, with no pass over the conv output or its gradient
# ---------------------------------------------------------------------------
BNRES = os.environ.get("SINGA_AMD_BNRES", "1") != "0"


def bnres_ok(y: torch.Tensor, w_shape, res: Optional[torch.Tensor], down=None) -> bool:
    """The fused residual tail applies: native bf16 channels_last, a 1x1 /
    stride-1 conv with C % 64 == 0 inputs and K4 % 128 == 0 outputs, a
    residual of the output's shape, non-deterministic mode.  ``down`` = (x,
    stride): instead of a residual, a strided 1x1 shortcut conv of x (C_x %
    64 == 0) onto the output grid (ConvBNDualAddReLU)."""
    K4, C = int(w_shape[0]), int(w_shape[1])
    ok = (BNRES and _native_ok(y) and y.dtype == torch.bfloat16 and N.is_cl(y) and y.dim() == 4
          and tuple(w_shape[2:]) == (1, 1) and y.shape[1] == C and C % 64 == 0 and K4 % 128 == 0
          and not N.lib().deterministic() and y.numel() // C * K4 * 2 < (1 << 31))
    if not ok:
        return False
    if down is not None:
        x, s = down
        return (_native_ok(x) and x.dtype == torch.bfloat16 and x.dim() == 4 and N.is_cl(x) and x.shape[1] % 64 == 0
                and x.shape[0] == y.shape[0] and (x.shape[2] - 1) // s + 1 == y.shape[2]
                and (x.shape[3] - 1) // s + 1 == y.shape[3] and x.numel() * 2 < (1 << 31))
    return res is not None and tuple(res.shape) == (y.shape[0], K4, y.shape[2], y.shape[3])


# the tail's forward recomputes its 1x1 conv instead of storing the output
# (bnres_fwd); switchable for A/B measurements
TAIL_RECOMPUTE = os.environ.get("SINGA_AMD_TAIL_RECOMPUTE", "1") != "0"
# ... and takes its BN statistics from Gram(y) and colsum(y) instead of a
# statistics-only GEMM pass (tail_stats_ws)
GRAM_STATS = os.environ.get("SINGA_AMD_GRAM_STATS", "1") != "0"


def tail_stats_ws(a: torch.Tensor, w: torch.Tensor, M: int, C: int, K4: int):
    """(ws, rows) for bn_fwd_from_ws: the per-channel sum and sum of squares of
    c = conv1x1(a, w) without computing c -- sum_k = W[k] . colsum(a),
    sumsq_k = W[k]^T Gram(a) W[k], Gram(a) = a^T a one K-outer GEMM over the
    pixels (a C x C output, split-K) -- or the statistics-only pass of the
    persistent GEMM (GRAM_STATS off).  colsum(a): the producer BN's apply-pass
    slot rows when it summed them (``_sg_cs_slots``), else one reduction."""
    L = N.lib()
    dev = a.device
    if not GRAM_STATS:
        ws = zeroed_ws(32 * 2 * K4, dev)
        L.sk_tail(a.data_ptr(), w.data_ptr(), 0, ws.data_ptr(), 0, 0, 0, 0, M, K4, C, 0, N.stream())
        return ws, 32
    gram = _zeros32(C * C, dev)
    L.bnres_wgrad(0, a.data_ptr(), gram.data_ptr(), M, 0, C, N.stream())
    cs = getattr(a, "_sg_cs_slots", None)
    if cs is None or cs.numel() % C != 0:
        cs = colsum(a.permute(0, 2, 3, 1).reshape(M, C))[0]
    ws = _mem.empty(2 * K4, dtype=torch.float32, device=dev)
    L.bnres_gram_stats(w.data_ptr(), gram.data_ptr(), cs.data_ptr(), cs.numel() // C, K4, C, ws.data_ptr(),
                       N.stream())
    return ws, 1


def bnres_fwd(y: torch.Tensor, w: torch.Tensor, gamma, beta, run_mean, run_var, training: bool, momentum: float,
              eps: float, res: torch.Tensor):
    """Training forward of the fused residual tail relu(BN(conv1x1(y, w)) +
    res) without materialising the conv output c: the persistent short-K GEMM
    runs twice -- once for the BN statistics only, once with the BN affine,
    the residual add, the ReLU and the mask bits in its epilogue.  On the
    short-K tails (stage 1/2: 64/128 input channels for 256/512 outputs) the
    second GEMM reads y again (K bf16 per row) where the unfused path writes
    and re-reads c (N bf16 per row each way): 4.2 vs 7.1 GB per stage-1 block
    at batch 1024.  Results are bitwise those of the unfused path (same
    statistics kernel, same bf16 rounding of c before the affine).  Returns
    (out, BNState) or None when the shape does not take the persistent kernel
    (the caller then runs conv + batchnorm_fwd)."""
    if not (TAIL_RECOMPUTE and training and _native_ok(y, w) and y.dtype == torch.bfloat16 and y.dim() == 4
            and N.is_cl(y) and tuple(w.shape[2:]) == (1, 1) and res is not None and res.dtype == torch.bfloat16
            and N.is_cl(res)):
        return None
    if not (w.dtype == torch.bfloat16 and N.is_cl(w)):
        w = G.to(w, torch.bfloat16, torch.channels_last)
    Nn, C, H, W = y.shape
    K = w.shape[0]
    M = Nn * H * W
    L = N.lib()
    if w.shape[1] != C or tuple(res.shape) != (Nn, K, H, W) or not L.sk_tail_ok(M, K, C):
        return None
    dev = y.device
    ws, rows = tail_stats_ws(y, w, M, C, K)
    p = _mem.empty(4 * K, dtype=torch.float32, device=dev)
    mean, invstd, scale, shift = p[:K], p[K:2 * K], p[2 * K:3 * K], p[3 * K:]
    L.bn_fwd_from_ws(ws.data_ptr(), rows, gamma.data_ptr(), beta.data_ptr(), run_mean.data_ptr(), run_var.data_ptr(),
                     mean.data_ptr(), invstd.data_ptr(), scale.data_ptr(), shift.data_ptr(), M, K, momentum, eps,
                     N.stream())
    out = _mem.empty((Nn, K, H, W), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    mask = _mem.empty(M * K // 8, dtype=torch.uint8, device=dev)
    L.sk_tail(y.data_ptr(), w.data_ptr(), out.data_ptr(), 0, scale.data_ptr(), shift.data_ptr(), res.data_ptr(),
              mask.data_ptr(), M, K, C, 1, N.stream())
    return out, BNState(mean, invstd, scale, shift, mask)


def bnres_dual_fwd(y, w3, g3, b3, rm3, rv3, mom3, eps3, x, wd, gd, bd, rmd, rvd, momd, epsd, training: bool):
    """Training forward of the two-branch (downsample, stride-1) tail
    relu(BN3(conv1x1(y, w3)) + BNd(conv1x1(x, wd))) with neither conv output
    stored: one statistics-only persistent-GEMM pass per branch, then ONE pass
    over the two-source operand [y | x] against both branches' weights with
    their BN scales folded in, BN shifts + ReLU + mask in the epilogue
    (sk_tail2; K = C_y + C_x <= 128: ResNet-50's stage-1 downsample block).
    Same statistics as the unfused path; the output differs only by the bf16
    rounding of the folded weights.  Returns (out, st3, std) or None."""
    if not (TAIL_RECOMPUTE and training and _native_ok(y, w3, x, wd) and y.dtype == torch.bfloat16
            and x.dtype == torch.bfloat16 and y.dim() == 4 and x.dim() == 4 and N.is_cl(y) and N.is_cl(x)
            and tuple(w3.shape[2:]) == (1, 1) and tuple(wd.shape[2:]) == (1, 1)):
        return None
    Nn, C1, H, W = y.shape
    C2 = x.shape[1]
    K4 = w3.shape[0]
    M = Nn * H * W
    L = N.lib()
    if (tuple(x.shape) != (Nn, C2, H, W) or w3.shape[1] != C1 or tuple(wd.shape[:2]) != (K4, C2) or C1 % 64 != 0
            or not L.sk_tail_ok(M, K4, C1 + C2) or not L.sk_tail_ok(M, K4, C1) or not L.sk_tail_ok(M, K4, C2)):
        return None
    to_b = lambda w: w if (w.dtype == torch.bfloat16 and N.is_cl(w)) else G.to(w, torch.bfloat16,  # noqa: E731
                                                                                 torch.channels_last)
    w3, wd = to_b(w3), to_b(wd)
    dev = y.device
    sts = []
    for a, w, g, b, rm, rv, mom, eps, C in ((y, w3, g3, b3, rm3, rv3, mom3, eps3, C1),
                                           (x, wd, gd, bd, rmd, rvd, momd, epsd, C2)):
        ws, rows = tail_stats_ws(a, w, M, C, K4)
        p = _mem.empty(4 * K4, dtype=torch.float32, device=dev)
        mean, invstd, scale, shift = p[:K4], p[K4:2 * K4], p[2 * K4:3 * K4], p[3 * K4:]
        L.bn_fwd_from_ws(ws.data_ptr(), rows, g.data_ptr(), b.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                         mean.data_ptr(), invstd.data_ptr(), scale.data_ptr(), shift.data_ptr(), M, K4, mom, eps,
                         N.stream())
        sts.append((mean, invstd, scale, shift))
    wf = _mem.empty(K4 * (C1 + C2), dtype=torch.bfloat16, device=dev)
    aux = _mem.empty(2 * K4, dtype=torch.float32, device=dev)
    L.bnres_fold(w3.data_ptr(), wd.data_ptr(), sts[0][2].data_ptr(), sts[0][3].data_ptr(), sts[1][2].data_ptr(),
                 sts[1][3].data_ptr(), K4, C1, C2, wf.data_ptr(), aux.data_ptr(), aux[K4:].data_ptr(), N.stream())
    out = _mem.empty((Nn, K4, H, W), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    mask = _mem.empty(M * K4 // 8, dtype=torch.uint8, device=dev)
    if not L.sk_tail2(y.data_ptr(), x.data_ptr(), wf.data_ptr(), aux.data_ptr(), aux[K4:].data_ptr(), out.data_ptr(),
                      mask.data_ptr(), M, K4, C1, C2, N.stream()):
        raise RuntimeError("bnres_dual_fwd: persistent kernel refused an eligible shape")
    return out, BNState(*sts[0], mask), BNState(*sts[1], None)


def strided_pick(x: torch.Tensor, stride: int) -> torch.Tensor:
    """x[:, :, ::s, ::s] as a dense channels_last bf16 tensor (native; the
    pixels a strided 1x1 conv reads)."""
    Nn, C, H, W = x.shape
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = _mem.empty((Nn, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    N.lib().strided_pick(x.data_ptr(), y.data_ptr(), Nn, H, W, C, Ho, Wo, stride, 0, N.stream())
    return y


def strided_place(xs: torch.Tensor, shape, stride: int) -> torch.Tensor:
    """The reverse of :func:`strided_pick`: a full-grid tensor of ``shape``
    with xs at every s-th pixel and zeros between (a strided 1x1 conv's input
    gradient)."""
    Nn, C, H, W = shape
    Ho, Wo = xs.shape[2], xs.shape[3]
    dx = _mem.empty((Nn, C, H, W), dtype=xs.dtype, device=xs.device, memory_format=torch.channels_last)
    N.lib().strided_pick(xs.data_ptr(), dx.data_ptr(), Nn, H, W, C, Ho, Wo, stride, 1, N.stream())
    dx._sg_fresh = True
    return dx


def _zeros32(n: int, device) -> torch.Tensor:
    """n zeroed fp32 (an arena slice when the step arena is active)."""
    t = ARENA.take(n, device)
    if t is None:
        t = _mem.empty(n, dtype=torch.float32, device=device)
        N.lib().zero(t.data_ptr(), 4 * n, N.stream())
    return t


def bnres_masksum(dy: torch.Tensor, mask: torch.Tensor):
    """g = dy * bit(mask) and the 32 slot rows of sum g (the fallback when no
    upstream dgrad epilogue produced them)."""
    if dy.dtype != torch.bfloat16 or not N.is_cl(dy):
        dy = G.to(dy, torch.bfloat16, torch.channels_last)
    C = dy.shape[1]
    R = dy.numel() // C
    g = _like(dy)
    ws = _zeros32(32 * 2 * C, dy.device)
    N.lib().bnres_masksum(dy.data_ptr(), mask.data_ptr(), g.data_ptr(), ws.data_ptr(), R, C, N.stream())
    return g, ws


def bnres_bwd(g: torch.Tensor, gws: torch.Tensor, y: torch.Tensor, w: torch.Tensor, st: "BNState",
              gamma: torch.Tensor, dw_out=None, dg_out=None, db_out=None, prod2=None, cs=None):
    """Backward of relu(BN(conv1x1(y, w)) + res) from g = d(out) * mask (bf16
    NHWC [N, K4, H, W]) and its per-channel sums (``gws``: 32 slot rows
    [32][2][K4]).  Returns (dy, dw, dgamma, dbeta); the parameter gradients
    accumulate into the *_out views when given.  ``prod2`` = (mask2, gamma2,
    beta2) of a producer BN(+ReLU) of y eligible for the identity-sum
    backward: the data gradient's epilogue then sums its masked output and
    the combination pass its <W, dW> sums (``dy._sg_bnbwd_wdot``), as
    conv2d_bwd's identity-sum path does."""
    L = N.lib()
    s = N.stream()
    dev = g.device
    Nn, K4, H, W = g.shape
    C = y.shape[1]
    P = Nn * H * W
    f32 = torch.float32
    wb = w if (w.dtype == torch.bfloat16 and (N.is_cl(w) or w.is_contiguous())) else G.to(w, torch.bfloat16)
    aug = _zeros32((K4 + C) * C, dev)  # [G ; Gram]
    L.bnres_wgrad(g.data_ptr(), y.data_ptr(), aug.data_ptr(), P, K4, C, s)
    Gm, Gram = aug[:K4 * C], aug[K4 * C:]
    coef = _mem.empty(3 * K4, dtype=f32, device=dev)
    wf = _mem.empty(K4 * C, dtype=f32, device=dev)
    wu = _mem.empty(K4 * C, dtype=f32, device=dev)
    dg = dg_out if dg_out is not None else _zeros32(K4, dev)
    db = db_out if db_out is not None else _zeros32(K4, dev)
    L.bnres_coef(Gm.data_ptr(), wb.data_ptr(), gws.data_ptr(), st.mean.data_ptr(), st.invstd.data_ptr(),
                 gamma.data_ptr(), P, K4, C, coef.data_ptr(), wf.data_ptr(), wu.data_ptr(), dg.data_ptr(),
                 db.data_ptr(), s)
    # the two small fp32 GEMMs accumulate (split-K atomics) into zeroed arena
    # slices: no zeroing launch of their own
    TM = _zeros32(K4 * C + C * C, dev)
    T, Mm = TM[:K4 * C], TM[K4 * C:]  # W Gram ; W^T diag(u) W
    L.ggemm(0, wf.data_ptr(), C, 0, 0, Gram.data_ptr(), C, 1, 0, T.data_ptr(), C, 0, K4, C, C, 1.0, 1.0, 0, 0, 2, 0,
            1, 0, 0, 0, 0, s)
    L.ggemm(0, wf.data_ptr(), C, 1, 0, wu.data_ptr(), C, 1, 0, Mm.data_ptr(), C, 0, C, C, K4, 1.0, 1.0, 0, 0, 2, 0,
            1, 0, 0, 0, 0, s)
    if cs is None:  # (the producer BN's apply pass sums them when it knows this consumer: st.colsum)
        cs = colsum(y.permute(0, 2, 3, 1).reshape(P, C))[0]
    cs_rows = cs.numel() // C  # 1, or the 32 slot rows of bn_apply_cs
    bd = _mem.empty(C * (K4 + C), dtype=torch.bfloat16, device=dev)
    bw = _zeros32(2 * C + 64, dev)
    wdot, bias = bw[:C + 1], bw[C + 64:]
    dw = dw_out if dw_out is not None else _zeros32(K4 * C, dev)
    g2, b2 = (prod2[1], prod2[2]) if prod2 is not None else (None, None)
    L.bnres_combine(Gm.data_ptr(), T.data_ptr(), Mm.data_ptr(), cs.data_ptr(), cs_rows, coef.data_ptr(), wb.data_ptr(), K4,
                    C, dw.data_ptr(), bd.data_ptr(), bias.data_ptr(), wdot.data_ptr(), N.ptr(g2), N.ptr(b2),
                    BN_WDOT_TAU, s)
    dy = _mem.empty((Nn, C, H, W), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    bws = _zeros32(32 * 2 * C, dev) if prod2 is not None else None
    L.bnres_dgrad(g.data_ptr(), y.data_ptr(), bd.data_ptr(), bias.data_ptr(), dy.data_ptr(), P, K4, C, N.ptr(bws),
                  N.ptr(prod2[0]) if prod2 is not None else 0, s)
    if prod2 is not None:
        dy._sg_bnbwd_wdot = (bws, wdot)
    dy._sg_fresh = True
    if dw_out is None:
        dw = dw.view(K4, C, 1, 1)
    return dy, dw, dg, db


def batchnorm_bwd(x: torch.Tensor, dy: torch.Tensor, gamma: torch.Tensor, st: BNState,
                  y_for_mask: Optional[torch.Tensor] = None, need_dres: bool = False, relu: bool = False,
                  dg_out: Optional[torch.Tensor] = None, db_out: Optional[torch.Tensor] = None,
                  beta: Optional[torch.Tensor] = None, lazy_dres: bool = False):
    """Returns dx, dgamma, dbeta, dres.  ReLU mask: from ``y_for_mask`` (the
    fused output, required when a residual was added) or, with ``relu`` and no
    residual, recomputed from x*scale+shift.  dgamma/dbeta are accumulated
    into dg_out/db_out when given (and those are returned).  ``lazy_dres``
    (native, 1-bit mask): dres is returned as a :class:`MaskedGrad` of dy
    instead of being written."""
    C = x.shape[1]
    if _bn_native(x):
        L = N.lib()
        R = x.numel() // C
        if dy.dtype != x.dtype or not _same_layout(dy, x):
            dy = G.to(dy, x.dtype, torch.channels_last if x.dim() == 4 else torch.contiguous_format)
        ym = y_for_mask
        if st.mask is not None and relu:
            ym, mode = st.mask, 3  # 1-bit mask written by the forward apply
        elif ym is not None:
            if ym.dtype != x.dtype or not _same_layout(ym, x):
                raise ValueError("batchnorm_bwd: mask tensor layout mismatch")
            mode = 1
        else:
            mode = 2 if relu else 0
        dg = dg_out if dg_out is not None else G.zeros((C,), torch.float32, x.device)
        db = db_out if db_out is not None else G.zeros((C,), torch.float32, x.device)
        coef = _mem.empty(3 * C, dtype=torch.float32, device=x.device)
        dx = _like(x)
        lazy = (need_dres and lazy_dres and LAZY_RES and mode == 3 and C % 8 == 0 and dy.dtype == torch.bfloat16
                and x.dtype == torch.bfloat16)
        dres = _like(x) if need_dres and not lazy else None
        wdot = getattr(dy, "_sg_bnbwd_wdot", None)  # identity-sum inputs from the consuming conv
        if (wdot is not None and mode == 3 and not need_dres and beta is not None and x.dtype == torch.bfloat16
                and C % 8 == 0 and dy.dtype == torch.bfloat16):
            ws2 = zeroed_ws(32 * 2 * C, x.device)
            flag = wdot[1][C:]  # raised by the conv's <W, dW> pass when gamma fails the recovery gate
            L.bn_bwd_wdot(x.data_ptr(), dy.data_ptr(), ym.data_ptr(), st.scale.data_ptr(), st.shift.data_ptr(),
                          st.mean.data_ptr(), st.invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                          wdot[0].data_ptr(), wdot[1].data_ptr(), ws2.data_ptr(), flag.data_ptr(), coef.data_ptr(),
                          dg.data_ptr(), db.data_ptr(), dx.data_ptr(), R, C, BN_WDOT_TAU, N.stream())
            dx._sg_fresh = True
            return dx, dg, db, None
        pre = getattr(dy, "_sg_bnbwd_ws", None)  # partial sums from the consuming conv's dgrad epilogue
        if pre is not None and ((mode == 2 and not need_dres) or mode == 3):
            L.bn_bwd_from_ws(x.data_ptr(), dy.data_ptr(), N.ptr(ym) if mode == 3 else 0, st.scale.data_ptr(),
                             st.shift.data_ptr(), st.mean.data_ptr(), st.invstd.data_ptr(), gamma.data_ptr(),
                             pre[0].data_ptr(), pre[1], coef.data_ptr(), dg.data_ptr(), db.data_ptr(), dx.data_ptr(),
                             N.ptr(dres), R, C, mode, N.dt(x), N.stream())
            dx._sg_fresh = True
            if dres is not None:
                dres._sg_fresh = True
            return dx, dg, db, (MaskedGrad(dy, ym) if lazy else dres)
        L.bn_bwd(x.data_ptr(), dy.data_ptr(), N.ptr(ym), st.scale.data_ptr(), st.shift.data_ptr(),
                 st.mean.data_ptr(), st.invstd.data_ptr(), gamma.data_ptr(), _ws(R, C, x.device).data_ptr(),
                 coef.data_ptr(), dg.data_ptr(), db.data_ptr(), dx.data_ptr(), N.ptr(dres), R, C, mode, N.dt(x),
                 N.stream())
        dx._sg_fresh = True
        if dres is not None:
            dres._sg_fresh = True
        return dx, dg, db, (MaskedGrad(dy, ym) if lazy else dres)
    _no_native("batchnorm_bwd", x, dy)
    if CP.ok(x, dy, gamma, y_for_mask, dg_out, db_out) and x.dim() in (2, 4):
        xc, dyc = CP.dense32(x), CP.dense32(dy)
        Nn = x.shape[0]
        HW = x.numel() // (Nn * C) if Nn * C else 0
        dg = dg_out if dg_out is not None and dg_out.is_contiguous() else G.zeros((C,), torch.float32, x.device)
        db = db_out if db_out is not None and db_out.is_contiguous() else G.zeros((C,), torch.float32, x.device)
        dx = _mem.empty(x.shape, dtype=torch.float32)
        dres = _mem.empty(x.shape, dtype=torch.float32) if need_dres else None
        ym = CP.dense32(y_for_mask) if y_for_mask is not None else None
        relu_x = int(relu and ym is None)
        CP.lib().bn_bwd(xc.data_ptr(), dyc.data_ptr(), CP.dense32(gamma).data_ptr(), CP.dense32(st.mean).data_ptr(),
                        CP.dense32(st.invstd).data_ptr(), CP.p(ym), relu_x,
                        CP.dense32(st.scale).data_ptr() if relu_x else 0,
                        CP.dense32(st.shift).data_ptr() if relu_x else 0, dx.data_ptr(), dg.data_ptr(), db.data_ptr(),
                        CP.p(dres), Nn, C, HW)
        if dg_out is not None and dg is not dg_out:
            dg = G.binary("add", dg_out, dg, out=dg_out)
            db = G.binary("add", db_out, db, out=db_out)
        return dx, dg, db, dres
    dims = (0,) if x.dim() == 2 else (0, 2, 3)
    shp = (1, C) if x.dim() == 2 else (1, C, 1, 1)
    g = dy.float()
    if y_for_mask is not None:
        g = g * (y_for_mask > 0)
    elif relu:
        g = g * ((x.float() * st.scale.reshape(shp) + st.shift.reshape(shp)) > 0)
    xh = (x.float() - st.mean.reshape(shp)) * st.invstd.reshape(shp)
    cnt = x.numel() // C
    sdy = g.sum(dims)
    sdyx = (g * xh).sum(dims)
    dx = gamma.float().reshape(shp) * st.invstd.reshape(shp) * (g - sdy.reshape(shp) / cnt -
                                                                  xh * sdyx.reshape(shp) / cnt)
    if dg_out is not None:
        dg_out.add_(sdyx)
        sdyx = dg_out
    if db_out is not None:
        db_out.add_(sdy)
        sdy = db_out
    return dx.to(x.dtype), sdyx, sdy, (g.to(x.dtype) if need_dres else None)


def pool2d_fwd(x: torch.Tensor, kernel, stride, padding, is_max: bool, count_include_pad: bool = True,
               ceil_mode: bool = False):
    kh, kw = kernel
    sh, sw = stride
    ph, pw = padding
    Nn, C, H, W = x.shape
    if ceil_mode:
        Ho = -(-(H + 2 * ph - kh) // sh) + 1
        Wo = -(-(W + 2 * pw - kw) // sw) + 1
    else:
        Ho = (H + 2 * ph - kh) // sh + 1
        Wo = (W + 2 * pw - kw) // sw + 1
    if _native_ok(x) and x.dtype in (torch.float32, torch.bfloat16):
        if kh * kw > 255 and is_max:
            raise NotImplementedError("max pool windows of more than 255 taps (8-bit argmax)")
        x = G.to(x, memory_format=torch.channels_last)
        y = _mem.empty((Nn, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        arg = _mem.empty((Nn, Ho, Wo, C), dtype=torch.uint8, device=x.device) if is_max else None
        N.lib().pool_fwd(x.data_ptr(), y.data_ptr(), N.ptr(arg), Nn, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw,
                         int(is_max), int(count_include_pad), N.dt(x), N.stream())
        return y, arg
    _no_native("pool2d_fwd", x)
    if CP.ok(x):
        xc = CP.dense32(x)
        y = _mem.empty((Nn, C, Ho, Wo), dtype=torch.float32)
        arg = _mem.empty((Nn, C, Ho, Wo), dtype=torch.int32) if is_max else None
        CP.lib().pool_fwd(xc.data_ptr(), y.data_ptr(), CP.p(arg), Nn, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw,
                          int(is_max), int(count_include_pad))
        return y, arg
    xf = x.float()
    if is_max:
        y, idx = F.max_pool2d(xf, (kh, kw), (sh, sw), (ph, pw), ceil_mode=ceil_mode, return_indices=True)
        return y.to(x.dtype), idx
    y = F.avg_pool2d(xf, (kh, kw), (sh, sw), (ph, pw), ceil_mode=ceil_mode, count_include_pad=count_include_pad)
    return y.to(x.dtype), None


def pool2d_bwd(x_shape, x_like: torch.Tensor, dy: torch.Tensor, arg, kernel, stride, padding, is_max: bool,
               count_include_pad: bool = True, ceil_mode: bool = False):
    kh, kw = kernel
    sh, sw = stride
    ph, pw = padding
    Nn, C, H, W = x_shape
    Ho, Wo = dy.shape[2], dy.shape[3]
    if _native_ok(dy) and dy.dtype in (torch.float32, torch.bfloat16):
        dy = G.to(dy, memory_format=torch.channels_last)
        dx = _mem.empty(x_shape, dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        N.lib().pool_bwd(dy.data_ptr(), N.ptr(arg), dx.data_ptr(), Nn, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw,
                         int(is_max), int(count_include_pad), N.dt(dy), N.stream())
        return dx
    _no_native("pool2d_bwd", dy)
    if CP.ok(dy) and (not is_max or arg.dtype == torch.int32):
        dyc = CP.dense32(dy)
        dx = _mem.empty(tuple(x_shape), dtype=torch.float32)
        a = G.contiguous(arg) if is_max else None
        CP.lib().pool_bwd(dyc.data_ptr(), CP.p(a), dx.data_ptr(), Nn, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw,
                          int(is_max), int(count_include_pad))
        return dx
    if is_max and arg.dtype != torch.int64:
        arg = arg.long()
    g = dy.float()
    if is_max:  # scatter-ADD: overlapping windows (k > s) may pick the same input
        dx = torch.zeros((Nn, C, H * W), dtype=torch.float32, device=dy.device)
        dx.scatter_add_(2, arg.reshape(Nn, C, -1), g.reshape(Nn, C, -1))
        return dx.view(Nn, C, H, W).to(dy.dtype)
    with torch.enable_grad():
        xx = torch.zeros(x_shape, dtype=torch.float32, device=dy.device, requires_grad=True)
        y = F.avg_pool2d(xx, (kh, kw), (sh, sw), (ph, pw), ceil_mode=ceil_mode, count_include_pad=count_include_pad)
        (dx,) = torch.autograd.grad(y, xx, g)
    return dx.to(dy.dtype)


def global_avgpool_fwd(x: torch.Tensor) -> torch.Tensor:
    Nn, C, H, W = x.shape
    if _native_ok(x) and x.dtype in (torch.float32, torch.bfloat16):
        x = G.to(x, memory_format=torch.channels_last)
        y = _mem.empty((Nn, C), dtype=x.dtype, device=x.device)
        N.lib().gap_fwd(x.data_ptr(), y.data_ptr(), Nn, H * W, C, N.dt(x), N.stream())
        return y
    _no_native("global_avgpool_fwd", x)
    if CP.ok(x):
        return G.reduce(x, [2, 3], "mean")
    return x.float().mean(dim=(2, 3)).to(x.dtype)


def global_avgpool_bwd(dy: torch.Tensor, x_shape) -> torch.Tensor:
    Nn, C, H, W = x_shape
    if _native_ok(dy) and dy.dtype in (torch.float32, torch.bfloat16):
        dy = G.contiguous(dy)
        dx = _mem.empty(x_shape, dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        N.lib().gap_bwd(dy.data_ptr(), dx.data_ptr(), Nn, H * W, C, N.dt(dy), N.stream())
        return dx
    _no_native("global_avgpool_bwd", dy)
    if CP.ok(dy):
        return G.expand(unary("scale", dy, 1.0 / (H * W)).reshape(Nn, C, 1, 1), tuple(x_shape))
    return (dy.float()[:, :, None, None] / (H * W)).expand(x_shape).to(dy.dtype)


def _lrn_rows_ok(x, size):
    C = x.shape[1]
    return C % 8 == 0 and C <= 2048 and size % 2 == 1 and size <= 9 and size <= C


def lrn_fwd(x: torch.Tensor, size: int, alpha: float, beta: float, k: float):
    """Returns (y, norm); norm is None on the pixel-staged native path
    (lrn_bwd then recomputes it from x and needs ``k``)."""
    if _native_ok(x) and x.dtype in (torch.float32, torch.bfloat16) and not N.is_cl(x):
        x = G.to(x, memory_format=torch.channels_last)
    if _native_ok(x) and _flat_ok(x) and N.is_cl(x) and _lrn_rows_ok(x, size):
        C = x.shape[1]
        y = _like(x)
        N.lib().lrn_rows(x.data_ptr(), 0, y.data_ptr(), x.numel() // C, C, size, alpha, beta, k, 0, N.dt(x),
                         N.stream())
        return y, None
    if _native_ok(x) and _flat_ok(x) and N.is_cl(x):
        C = x.shape[1]
        R = x.numel() // C
        y = _like(x)
        norm = _mem.empty(x.shape, dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
        N.lib().lrn_fwd(x.data_ptr(), y.data_ptr(), norm.data_ptr(), R, C, size, alpha, beta, k, N.dt(x),
                        N.stream())
        return y, norm
    _no_native("lrn_fwd", x)
    if CP.ok(x) and x.dim() == 4:
        xc = CP.dense32(x)
        Nn, C, H, W = x.shape
        y = _mem.empty(x.shape, dtype=torch.float32)
        CP.lib().lrn_fwd(xc.data_ptr(), y.data_ptr(), Nn, C, H * W, int(size), float(alpha), float(beta), float(k))
        return y, None  # the backward recomputes the window sums
    xf = x.float()
    sq = xf * xf
    half = size // 2
    pad = F.pad(sq, (0, 0, 0, 0, half, half))
    s = sum(pad[:, i:i + x.shape[1]] for i in range(size))
    norm = k + alpha / size * s
    return (xf * norm.pow(-beta)).to(x.dtype), norm


def lrn_bwd(x: torch.Tensor, dy: torch.Tensor, norm: Optional[torch.Tensor], size: int, alpha: float, beta: float,
            k: float = 1.0, relu_mask: bool = False):
    """``relu_mask``: x is a ReLU output; the native kernel also zeroes dx
    where x <= 0 (the ReLU backward, folded) and marks dx ``_sg_relu_done``."""
    if CP.ok(x, dy) and x.dim() == 4:
        xc, dyc = CP.dense32(x), CP.dense32(dy)
        Nn, C, H, W = x.shape
        dx = _mem.empty(x.shape, dtype=torch.float32)
        CP.lib().lrn_bwd(xc.data_ptr(), dyc.data_ptr(), dx.data_ptr(), Nn, C, H * W, int(size), float(alpha),
                         float(beta), float(k))
        return dx
    if _native_ok(x, dy) and x.dtype in (torch.float32, torch.bfloat16):
        x = G.to(x, memory_format=torch.channels_last)
        dy = G.to(dy, x.dtype, torch.channels_last)
    if norm is None:  # pixel-staged forward: recompute norm from x inside the backward kernel
        if (_native_ok(x, dy) and _flat_ok(x) and N.is_cl(x) and N.is_cl(dy) and dy.dtype == x.dtype
                and _lrn_rows_ok(x, size)):
            C = x.shape[1]
            dx = _like(x)
            dyc = dy if dy.is_contiguous(memory_format=torch.channels_last) else dy.contiguous(
                memory_format=torch.channels_last)
            N.lib().lrn_rows(x.data_ptr(), dyc.data_ptr(), dx.data_ptr(), x.numel() // C, C, size, alpha, beta, k,
                             2 if relu_mask else 1, N.dt(x), N.stream())
            if relu_mask:
                dx._sg_relu_done = True
            return dx
        _no_native("lrn_bwd (window)", x)
        xf = x.float()
        half = size // 2
        s2 = sum(F.pad(xf * xf, (0, 0, 0, 0, half, half))[:, i:i + x.shape[1]] for i in range(size))
        norm = k + alpha / size * s2
    if _native_ok(x, dy) and _flat_ok(x) and N.is_cl(x) and N.is_cl(dy) and dy.dtype == x.dtype:
        C = x.shape[1]
        R = x.numel() // C
        dx = _like(x)
        N.lib().lrn_bwd(x.data_ptr(), dy.data_ptr(), norm.data_ptr(), dx.data_ptr(), R, C, size, alpha, beta,
                        N.dt(x), N.stream())
        return dx
    _no_native("lrn_bwd", x, dy)
    xf, g = x.float(), dy.float()
    t = g * xf * norm.pow(-beta - 1)
    half = size // 2
    pad = F.pad(t, (0, 0, 0, 0, half, half))
    s = sum(pad[:, i:i + x.shape[1]] for i in range(size))
    dx = g * norm.pow(-beta) - 2 * beta * alpha / size * xf * s
    return dx.to(dy.dtype)


# ---------------------------------------------------------------- attention
def attention_fwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, mask: Optional[torch.Tensor] = None,
                  scale: Optional[float] = None):
    """softmax(q k^T * scale + mask) v for q [..., Sq, D], k/v [..., Sk, D];
    mask broadcastable to [..., Sq, Sk] (additive).  Returns (o, p) with the
    probabilities p kept for backward.  GPU: batched MFMA GEMMs (bf16 or
    exact fp32, any head size / length) + the softmax kernels."""
    D = q.shape[-1]
    scale = (1.0 / math.sqrt(D)) if scale is None else scale
    lead = q.shape[:-2]
    Sq, Sk = q.shape[-2], k.shape[-2]
    if _native_ok(q, k, v) or CP.ok(q, k, v, mask):
        q3 = G.reshape(q, (-1, Sq, D))
        k3 = G.reshape(k, (-1, Sk, D))
        v3 = G.reshape(v, (-1, Sk, D))
        B = q3.shape[0]
        s = gemm(q3, k3, tb=True, alpha=scale, out_dtype=torch.float32)
        if mask is not None:
            s = G.binary("add", s.view(*lead, Sq, Sk), mask, out_dtype=torch.float32).reshape(B, Sq, Sk)
        p = softmax(s, out_dtype=q.dtype)
        o = gemm(p, v3, out_dtype=q.dtype)
        return o.view(*lead, Sq, D), p.view(*lead, Sq, Sk)
    _no_native("attention_fwd", q, k, v)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if mask is not None:
        s = s + mask.float()
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, v.float())
    return o.to(q.dtype), p.to(q.dtype)


def _gemm_heads(a, lda, ako, b, ldb, bko, c, ldc, M, Nn, K, batch, bh, sa, sa2, sb, sb2, sc, sc2, alpha=1.0):
    """Batched MFMA GEMM over (batch / bh, batch % bh) with two-level strides:
    a, b, c are (tensor, element offset) pairs -- attention heads addressed in
    place inside the [B, S, 3, H, D] projection / [B, S, H, D] output."""
    (ta, oa), (tb, ob), (tc, oc) = a, b, c
    mode = 0 if tc.dtype == torch.bfloat16 else 1
    N.lib().gemm_heads(ta.data_ptr() + 2 * oa, lda, ako, tb.data_ptr() + 2 * ob, ldb, bko,
                       tc.data_ptr() + tc.element_size() * oc, ldc, M, Nn, K, alpha, 0.0, mode, batch, sa, sb, sc,
                       bh, sa2, sb2, sc2, N.stream())


def _qkv_native_ok(qkv, H):
    if not (_native_ok(qkv) and qkv.dtype == torch.bfloat16 and qkv.dim() == 3 and qkv.is_contiguous()):
        return False
    B, S, E = qkv.shape
    return E % (3 * H) == 0 and (E // (3 * H)) % 8 == 0 and S % 8 == 0


class FAttnState:
    """What the fused attention backward needs from its forward: the per-row
    log-sum-exp, the output and the key mask (the probabilities are
    recomputed, never stored)."""

    __slots__ = ("lse", "o", "mask", "mstride")

    def __init__(self, lse, o, mask, mstride):
        self.lse, self.o, self.mask, self.mstride = lse, o, mask, mstride


def _fattn_mask(mask: Optional[torch.Tensor], B: int, S: int):
    """(mask tensor, batch stride) when ``mask`` is an additive key mask the
    fused kernel takes ([B or 1, 1, 1, S] or [B or 1, S], fp32, unit key
    stride, 16-byte aligned rows); (None, 0) for no mask; False otherwise."""
    if mask is None:
        return None, 0
    m = mask
    if m.dtype != torch.float32 or not m.is_cuda or m.shape[-1] != S or m.stride(-1) != 1:
        return False
    if m.dim() == 4 and (m.shape[1] != 1 or m.shape[2] != 1):
        return False
    if m.dim() not in (2, 4) or m.shape[0] not in (1, B):
        return False
    ms = m.stride(0) if m.shape[0] == B and B > 1 else 0
    if m.data_ptr() % 16 or (ms * 4) % 16:
        return False
    return m, ms


def _fattn_on() -> bool:
    return os.environ.get("SINGA_AMD_FATTN", "1") != "0"


def attention_qkv_fwd(qkv: torch.Tensor, heads: int, mask: Optional[torch.Tensor] = None,
                      scale: Optional[float] = None):
    """Multi-head attention straight from the fused projection: qkv [B, S,
    3*H*D] (per token: q heads, k heads, v heads) -> o [B, S, H*D] (heads
    merged), p [B*H, S, S] (bf16 probabilities, kept for backward).  The
    batched GEMMs address every (b, h) slice in place -- no split-heads /
    merge-heads copies in either direction."""
    B, S, E = qkv.shape
    H = heads
    D = E // (3 * H)
    HD = H * D
    scale = (1.0 / math.sqrt(D)) if scale is None else scale
    if _qkv_native_ok(qkv, H) and _fattn_on() and N.lib().fattn_ok(S, D):
        mk = _fattn_mask(mask, B, S)
        if mk is not False:
            # fused kernel (csrc/kernels/fattn.hip): QK^T, softmax and PV per
            # (batch, head) in registers / LDS; only the row log-sum-exp is kept
            m, ms = mk
            o = _mem.empty((B, S, HD), dtype=torch.bfloat16, device=qkv.device)
            lse = _mem.empty((B * H, S), dtype=torch.float32, device=qkv.device)
            N.lib().fattn_fwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), N.ptr(m), ms, B, S, H, D, scale,
                              N.stream())
            return o, FAttnState(lse, o, m, ms)
    if _qkv_native_ok(qkv, H):
        BH = B * H
        sc = _mem.empty((BH, S, S), dtype=torch.float32, device=qkv.device)
        # scores = q k^T * scale : q [S][D] rows of stride E, k [S][D] (N x K, K-major)
        _gemm_heads((qkv, 0), E, 0, (qkv, HD), E, 0, (sc, 0), S, S, S, D, BH, H, S * E, D, S * E, D, H * S * S,
                    S * S, alpha=scale)
        if mask is not None:
            sc = G.binary("add", sc.view(B, H, S, S), mask, out_dtype=torch.float32).reshape(BH, S, S)
        p = softmax(sc, out_dtype=torch.bfloat16)
        o = _mem.empty((B, S, HD), dtype=torch.bfloat16, device=qkv.device)
        # o = p v : v [S][D] is K-outer (ldb E); o rows of stride H*D
        _gemm_heads((p, 0), S, 0, (qkv, 2 * HD), E, 1, (o, 0), HD, S, D, S, BH, H, H * S * S, S * S, S * E, D,
                    S * HD, D)
        return o, p
    t = qkv.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
    o, p = attention_fwd(t[0], t[1], t[2], mask, scale)
    return G.reshape(G.contiguous(o.permute(0, 2, 1, 3)), (B, S, HD)), G.reshape(p, (B * H, S, S))


def fattn_bias_ok(p, db: Optional[torch.Tensor], E: int) -> bool:
    """The fused attention backward can sum d(qkv)'s columns into ``db``."""
    return (isinstance(p, FAttnState) and db is not None and db.is_cuda and db.dtype == torch.float32
            and db.is_contiguous() and db.numel() == E)


def attention_qkv_bwd(qkv: torch.Tensor, p: torch.Tensor, do: torch.Tensor, heads: int,
                      scale: Optional[float] = None, db_acc: Optional[torch.Tensor] = None) -> torch.Tensor:
    """d(qkv) [B, S, 3*H*D] of :func:`attention_qkv_fwd` given do [B, S, H*D];
    dq / dk / dv are written in place into their slots of d(qkv).
    ``db_acc`` (fp32 [3*H*D], fused path only: see :func:`fattn_bias_ok`)
    += the column sums of d(qkv), summed by the fused backward kernel."""
    B, S, E = qkv.shape
    H = heads
    D = E // (3 * H)
    HD = H * D
    scale = (1.0 / math.sqrt(D)) if scale is None else scale
    if isinstance(p, FAttnState):
        do = G.contiguous(G.to(do, torch.bfloat16))
        dqkv = _mem.empty_like(qkv)
        if db_acc is not None and not fattn_bias_ok(p, db_acc, E):
            raise ValueError("attention_qkv_bwd: db_acc must be a dense fp32 [3*H*D] device tensor")
        N.lib().fattn_bwd(qkv.data_ptr(), p.o.data_ptr(), do.data_ptr(), p.lse.data_ptr(), N.ptr(p.mask), p.mstride,
                          dqkv.data_ptr(), N.ptr(db_acc), B, S, H, D, scale, N.stream())
        return dqkv
    if db_acc is not None:
        raise ValueError("attention_qkv_bwd: db_acc needs the fused attention state")
    if _qkv_native_ok(qkv, H) and p.dtype == torch.bfloat16 and do.dtype == torch.bfloat16:
        BH = B * H
        do = G.contiguous(do)
        dqkv = _mem.empty_like(qkv)
        SS = S * S
        # dV = P^T dO
        _gemm_heads((p, 0), S, 1, (do, 0), HD, 1, (dqkv, 2 * HD), E, S, D, S, BH, H, H * SS, SS, S * HD, D, S * E, D)
        # dP = dO V^T
        dp = _mem.empty((BH, S, S), dtype=torch.bfloat16, device=qkv.device)
        _gemm_heads((do, 0), HD, 0, (qkv, 2 * HD), E, 0, (dp, 0), S, S, S, D, BH, H, S * HD, D, S * E, D, H * SS,
                    SS)
        ds = softmax_bwd(p, dp)
        # dQ = scale * dS K ; dK = scale * dS^T Q
        _gemm_heads((ds, 0), S, 0, (qkv, HD), E, 1, (dqkv, 0), E, S, D, S, BH, H, H * SS, SS, S * E, D, S * E, D,
                    alpha=scale)
        _gemm_heads((ds, 0), S, 1, (qkv, 0), E, 1, (dqkv, HD), E, S, D, S, BH, H, H * SS, SS, S * E, D, S * E, D,
                    alpha=scale)
        return dqkv
    t = qkv.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
    dq, dk, dv = attention_bwd(t[0], t[1], t[2], G.reshape(p, (B, H, S, S)),
                               G.reshape(do, (B, S, H, D)).permute(0, 2, 1, 3), scale)
    st = G.cat([dq.unsqueeze(0), dk.unsqueeze(0), dv.unsqueeze(0)], 0)  # [3, B, H, S, D]
    return G.to(G.reshape(G.contiguous(st.permute(1, 3, 0, 2, 4)), (B, S, E)), qkv.dtype)


def attention_bwd(q, k, v, p, do, scale: Optional[float] = None):
    """Gradients (dq, dk, dv) of attention_fwd given the saved probabilities."""
    D = q.shape[-1]
    scale = (1.0 / math.sqrt(D)) if scale is None else scale
    Sq, Sk = q.shape[-2], k.shape[-2]
    if _native_ok(q, k, v, p, do) or CP.ok(q, k, v, p, do):
        q3 = G.reshape(q, (-1, Sq, D))
        k3 = G.reshape(k, (-1, Sk, D))
        v3 = G.reshape(v, (-1, Sk, D))
        p3 = G.reshape(p, (-1, Sq, Sk))
        do3 = G.reshape(G.to(do, q.dtype), (-1, Sq, D))
        # dV = P^T dO ; dP = dO V^T ; dS = P * (dP - rowsum(dP * P)) ; dQ = scale dS K ; dK = scale dS^T Q
        dv = gemm(p3, do3, ta=True, out_dtype=v.dtype)
        dp = gemm(do3, v3, tb=True, out_dtype=p.dtype)
        ds = softmax_bwd(p3, dp)
        dq = gemm(ds, k3, alpha=scale, out_dtype=q.dtype)
        dk = gemm(ds, q3, ta=True, alpha=scale, out_dtype=k.dtype)
        return dq.view(q.shape), dk.view(k.shape), dv.view(v.shape)
    _no_native("attention_bwd", q, k, v)
    pf, dof = p.float(), do.float()
    dv = torch.matmul(pf.transpose(-1, -2), dof)
    dp = torch.matmul(dof, v.float().transpose(-1, -2))
    ds = pf * (dp - (dp * pf).sum(-1, keepdim=True))
    dq = torch.matmul(ds, k.float()) * scale
    dk = torch.matmul(ds.transpose(-1, -2), q.float()) * scale
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)
