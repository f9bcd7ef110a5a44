"""sonnx -- ONNX import / export for singa_amd (the SINGA ``sonnx`` API:
``to_onnx``, ``prepare`` / ``SingaBackend`` / ``SingaRep``, ``SONNXModel``).

Export traces one forward pass of a model (every autograd operator records
its inputs/outputs while :func:`to_onnx` runs) and lowers each operator to
ONNX nodes (opset 17); parameters become initializers named by their model
path, activations are exported as fp32 (bf16 casts become identities).

Import parses the protobuf (no ``onnx`` package, no code execution), turns
float initializers into trainable parameters, and executes the nodes in
order through the same autograd operators and HIP kernels as hand-built
models -- so an imported model can be fine-tuned (``SONNXModel``).

The reference snapshot has no ONNX support (SURVEY §5.4 lists it as a
north-star addition), so parity with it is unpinned; tests round-trip models
through export -> serialize -> import and compare outputs.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import autograd, model
from ..ops import functional as F
from ..tensor import Tensor
from . import onnx_proto as P

OPSET = 17

_NP2ONNX = {np.dtype(np.float32): P.FLOAT, np.dtype(np.float64): P.DOUBLE, np.dtype(np.int64): P.INT64,
            np.dtype(np.int32): P.INT32, np.dtype(np.uint8): P.UINT8, np.dtype(np.int8): P.INT8,
            np.dtype(np.bool_): P.BOOL, np.dtype(np.float16): P.FLOAT16, np.dtype(np.int16): P.INT16}
_ONNX2NP = {v: k for k, v in _NP2ONNX.items()}
_T2ONNX = {torch.float32: P.FLOAT, torch.bfloat16: P.FLOAT, torch.float16: P.FLOAT16, torch.int64: P.INT64,
           torch.int32: P.INT32, torch.uint8: P.UINT8, torch.bool: P.BOOL, torch.float64: P.DOUBLE}


# ----------------------------------------------------------------- helpers
def numpy_to_tensorproto(a: np.ndarray, name: str = ""):
    a = np.asarray(a)
    if a.dtype == np.float64:
        a = a.astype(np.float32)
    t = P.new("TensorProto")
    t.name = name
    t.dims.extend(a.shape)
    t.data_type = _NP2ONNX[a.dtype]
    t.raw_data = np.ascontiguousarray(a).tobytes()
    return t


def tensorproto_to_numpy(t) -> np.ndarray:
    dt = _ONNX2NP.get(t.data_type)
    if t.data_type == P.BFLOAT16:
        raw = np.frombuffer(t.raw_data, np.uint16).astype(np.uint32) << 16
        return raw.view(np.float32).reshape(tuple(t.dims))
    if dt is None:
        raise NotImplementedError(f"ONNX tensor data_type {t.data_type}")
    shape = tuple(t.dims)
    if t.raw_data:
        return np.frombuffer(t.raw_data, dtype=dt).reshape(shape).copy()
    if t.data_type in (P.FLOAT,):
        return np.asarray(t.float_data, np.float32).reshape(shape)
    if t.data_type in (P.INT64,):
        return np.asarray(t.int64_data, np.int64).reshape(shape)
    if t.data_type in (P.DOUBLE,):
        return np.asarray(t.double_data, np.float64).reshape(shape)
    if t.data_type == P.FLOAT16:
        return np.asarray(t.int32_data, np.uint16).view(np.float16).reshape(shape)
    return np.asarray(t.int32_data, dtype=dt).reshape(shape)


def make_attribute(name: str, v):
    a = P.new("AttributeProto")
    a.name = name
    if isinstance(v, bool):
        v = int(v)
    if isinstance(v, (int, np.integer)):
        a.type, a.i = P.A_INT, int(v)
    elif isinstance(v, (float, np.floating)):
        a.type, a.f = P.A_FLOAT, float(v)
    elif isinstance(v, str):
        a.type, a.s = P.A_STRING, v.encode()
    elif isinstance(v, np.ndarray):
        a.type = P.A_TENSOR
        a.t.CopyFrom(numpy_to_tensorproto(v))
    elif isinstance(v, (list, tuple)):
        if all(isinstance(x, (int, np.integer)) for x in v):
            a.type = P.A_INTS
            a.ints.extend(int(x) for x in v)
        elif all(isinstance(x, (int, float, np.number)) for x in v):
            a.type = P.A_FLOATS
            a.floats.extend(float(x) for x in v)
        else:
            a.type = P.A_STRINGS
            a.strings.extend(str(x).encode() for x in v)
    else:
        raise TypeError(f"attribute {name}: unsupported value {v!r}")
    return a


def make_node(op_type: str, inputs: Sequence[str], outputs: Sequence[str], name: str = "", **attrs):
    n = P.new("NodeProto")
    n.op_type, n.name = op_type, name
    n.input.extend(inputs)
    n.output.extend(outputs)
    for k, v in attrs.items():
        if v is not None:
            n.attribute.append(make_attribute(k, v))
    return n


def attr_value(a):
    t = a.type
    if t == P.A_FLOAT:
        return a.f
    if t == P.A_INT:
        return a.i
    if t == P.A_STRING:
        return a.s.decode()
    if t == P.A_TENSOR:
        return tensorproto_to_numpy(a.t)
    if t == P.A_FLOATS:
        return list(a.floats)
    if t == P.A_INTS:
        return list(a.ints)
    if t == P.A_STRINGS:
        return [s.decode() for s in a.strings]
    if t == P.A_GRAPH:
        return a.g
    raise NotImplementedError(f"attribute type {t}")


def _value_info(name: str, shape, elem=P.FLOAT, dynamic_batch: bool = False):
    v = P.new("ValueInfoProto")
    v.name = name
    v.type.tensor_type.elem_type = elem
    for i, d in enumerate(shape):
        dim = v.type.tensor_type.shape.dim.add()
        if dynamic_batch and i == 0:
            dim.dim_param = "batch"
        else:
            dim.dim_value = int(d)
    return v


# ================================================================== export
class _ExportCtx:
    def __init__(self, param_names: Dict[int, str]):
        self.names: Dict[int, str] = {}
        self.keep: List[object] = []
        self.nodes: List = []
        self.inits: "OrderedDict[str, np.ndarray]" = OrderedDict()
        self.param_names = param_names
        self.state_by_ptr: Dict[int, str] = {}
        self.const_names: set = set()  # initializers that are constants, not parameters (tagged on export)
        self.k = 0

    def fresh(self, base: str = "t") -> str:
        self.k += 1
        return f"{base}_{self.k}"

    def const(self, a: np.ndarray, base: str = "const") -> str:
        n = self.fresh(base)
        self.inits[n] = np.asarray(a)
        self.const_names.add(n)
        return n

    def named_const(self, t: torch.Tensor, fallback: str) -> str:
        """Initializer for a raw state tensor (BN running stats): its model
        state name when known, else ``fallback``."""
        n = self.state_by_ptr.get(t.data_ptr()) or fallback
        if n in self.inits:
            return n
        self.inits[n] = t.detach().float().cpu().numpy()
        self.const_names.add(n)
        return n

    def name_of(self, t: Tensor) -> str:
        n = self.names.get(id(t))
        if n is not None:
            return n
        # a leaf we have not seen: parameter or constant -> initializer
        if id(t) in self.param_names:
            n = self.param_names[id(t)]
        else:
            n = self.fresh("const")
            self.const_names.add(n)
        a = t.data.detach()
        if a.dtype == torch.bfloat16:
            a = a.float()
        self.inits[n] = a.cpu().numpy()
        self.names[id(t)] = n
        self.keep.append(t)
        return n

    def add(self, op_type, inputs, outputs, **attrs):
        self.nodes.append(make_node(op_type, inputs, outputs, name=self.fresh(op_type), **attrs))


_EXPORTERS = {}


def exporter(*cls_names):
    def deco(fn):
        for c in cls_names:
            _EXPORTERS[c] = fn
        return fn
    return deco


_UNARY = {"ReLU": "Relu", "Sigmoid": "Sigmoid", "Tanh": "Tanh", "SoftPlus": "Softplus", "Exp": "Exp", "Log": "Log",
          "Abs": "Abs", "Sqrt": "Sqrt", "Reciprocal": "Reciprocal", "Negative": "Neg", "Sign": "Sign",
          "Identity": "Identity", "SeLU": "Selu", "ToChannelsLast": "Identity", "InputPrep": "Identity",
          "Dropout": "Identity"}


@exporter(*_UNARY)
def _x_unary(c, op, xs, i, o):
    c.add(_UNARY[type(op).__name__], [i[0]], [o[0]])


@exporter("LeakyRelu", "Elu")
def _x_alpha(c, op, xs, i, o):
    c.add(type(op).__name__, [i[0]], [o[0]], alpha=float(op.alpha))


@exporter("Square")
def _x_square(c, op, xs, i, o):
    c.add("Mul", [i[0], i[0]], [o[0]])


@exporter("STanh")
def _x_stanh(c, op, xs, i, o):
    a, b = c.fresh(), c.fresh()
    c.add("Mul", [i[0], c.const(np.float32(0.6666667))], [a])
    c.add("Tanh", [a], [b])
    c.add("Mul", [b, c.const(np.float32(1.7159))], [o[0]])


@exporter("Gelu")
def _x_gelu(c, op, xs, i, o):
    a, b, d, e = c.fresh(), c.fresh(), c.fresh(), c.fresh()
    c.add("Div", [i[0], c.const(np.float32(math.sqrt(2.0)))], [a])
    c.add("Erf", [a], [b])
    c.add("Add", [b, c.const(np.float32(1.0))], [d])
    c.add("Mul", [i[0], d], [e])
    c.add("Mul", [e, c.const(np.float32(0.5))], [o[0]])


@exporter("Add")
def _x_add(c, op, xs, i, o):
    if getattr(op, "relu", False):
        t = c.fresh()
        c.add("Add", i[:2], [t])
        c.add("Relu", [t], [o[0]])
    else:
        c.add("Add", i[:2], [o[0]])


for _n, _t in (("Sub", "Sub"), ("Mul", "Mul"), ("Div", "Div"), ("Pow", "Pow"), ("Matmul", "MatMul"),
               ("AddBias", "Add")):
    def _mk(t):
        def f(c, op, xs, i, o):
            c.add(t, i[:2], [o[0]])
        return f
    _EXPORTERS[_n] = _mk(_t)


@exporter("Linear")
def _x_linear(c, op, xs, i, o):
    act = getattr(op, "act", None)  # a fused output activation exports as its own node(s)
    out = c.fresh() if act else o[0]
    if len(i) > 2:
        t = c.fresh()
        c.add("MatMul", i[:2], [t])
        c.add("Add", [t, i[2]], [out])
    else:
        c.add("MatMul", i[:2], [out])
    if act == "stanh":
        _x_stanh(c, op, xs, [out], o)
    elif act == "gelu":
        _x_gelu(c, op, xs, [out], o)
    elif act:
        if act not in ("relu", "sigmoid", "tanh"):
            raise NotImplementedError(f"sonnx export: Linear with fused {act}")
        c.add({"relu": "Relu", "sigmoid": "Sigmoid", "tanh": "Tanh"}[act], [out], [o[0]])


@exporter("Conv2d")
def _x_conv(c, op, xs, i, o):
    ph, pw = op.padding
    W = xs[1]
    out = c.fresh() if op.fuse_relu else o[0]
    c.add("Conv", i[:3] if op.has_bias else i[:2], [out], kernel_shape=list(W.shape[2:]),
          strides=list(op.stride), pads=[ph, pw, ph, pw], dilations=list(op.dilation), group=int(op.group))
    if op.fuse_relu:
        c.add("Relu", [out], [o[0]])


@exporter("BatchNorm2d")
def _x_bn(c, op, xs, i, o):
    base = i[1].rsplit(".", 1)[0] if "." in i[1] else i[1]
    rm = c.named_const(op.rm, base + ".running_mean")
    rv = c.named_const(op.rv, base + ".running_var")
    y = c.fresh() if (op.relu or op.has_residual) else o[0]
    c.add("BatchNormalization", [i[0], i[1], i[2], rm, rv], [y], epsilon=float(op.eps),
          momentum=float(1.0 - op.momentum))
    if op.has_residual:
        z = c.fresh() if op.relu else o[0]
        c.add("Add", [y, i[3]], [z])
        y = z
    if op.relu:
        c.add("Relu", [y], [o[0]])


@exporter("Pooling2d")
def _x_pool(c, op, xs, i, o):
    ph, pw = op.padding
    kw = dict(kernel_shape=list(op.kernel), strides=list(op.stride), pads=[ph, pw, ph, pw], ceil_mode=int(op.ceil))
    if op.is_max:
        c.add("MaxPool", [i[0]], [o[0]], **kw)
    else:
        c.add("AveragePool", [i[0]], [o[0]], count_include_pad=int(op.cip), **kw)


@exporter("GlobalAveragePool")
def _x_gap(c, op, xs, i, o):
    if op.keepdims:
        c.add("GlobalAveragePool", [i[0]], [o[0]])
    else:
        t = c.fresh()
        c.add("GlobalAveragePool", [i[0]], [t])
        c.add("Flatten", [t], [o[0]], axis=1)


@exporter("LRN")
def _x_lrn(c, op, xs, i, o):
    c.add("LRN", [i[0]], [o[0]], size=int(op.size), alpha=float(op.alpha), beta=float(op.beta), bias=float(op.k))


@exporter("SoftMax")
def _x_softmax(c, op, xs, i, o):
    c.add("Softmax", [i[0]], [o[0]], axis=int(op.axis))


@exporter("LayerNorm")
def _x_ln(c, op, xs, i, o):
    c.add("LayerNormalization", i[:3], [o[0]], axis=-1, epsilon=float(op.eps))


@exporter("Cast")
def _x_cast(c, op, xs, i, o):
    to = _T2ONNX.get(op.to, P.FLOAT)
    if op.to in (torch.bfloat16, torch.float32, torch.float16):  # exported graphs are fp32
        c.add("Identity", [i[0]], [o[0]])
    else:
        c.add("Cast", [i[0]], [o[0]], to=int(to))


@exporter("Reshape")
def _x_reshape(c, op, xs, i, o):
    shape = list(op.shape)
    if len(shape) > 1 and len(xs[0].shape) > 1 and shape[0] == xs[0].shape[0]:
        shape[0] = 0  # keep the batch dim symbolic ("copy from input")
    c.add("Reshape", [i[0], c.const(np.asarray(shape, np.int64))], [o[0]])


@exporter("Flatten")
def _x_flatten(c, op, xs, i, o):
    c.add("Flatten", [i[0]], [o[0]], axis=int(op.axis))


@exporter("Attention")
def _x_attention(c, op, xs, i, o):
    D = xs[0].shape[-1]
    scale = op.scale if op.scale is not None else 1.0 / math.sqrt(D)
    nd = len(xs[0].shape)
    perm = list(range(nd - 2)) + [nd - 1, nd - 2]
    kt, s, ss, p = c.fresh(), c.fresh(), c.fresh(), c.fresh()
    c.add("Transpose", [i[1]], [kt], perm=perm)
    c.add("MatMul", [i[0], kt], [s])
    c.add("Mul", [s, c.const(np.float32(scale))], [ss])
    if len(i) > 3:
        sm = c.fresh()
        c.add("Add", [ss, i[3]], [sm])
        ss = sm
    c.add("Softmax", [ss], [p], axis=-1)
    c.add("MatMul", [p, i[2]], [o[0]])


@exporter("SplitHeads")
def _x_split_heads(c, op, xs, i, o):
    B, S, E3 = xs[0].shape
    H = op.h
    D = E3 // (3 * H)
    r, t = c.fresh(), c.fresh()
    c.add("Reshape", [i[0], c.const(np.asarray([0, 0, 3, H, D], np.int64))], [r])
    c.add("Transpose", [r], [t], perm=[2, 0, 3, 1, 4])
    parts = [c.fresh() for _ in range(3)]
    c.add("Split", [t, c.const(np.asarray([1, 1, 1], np.int64))], parts, axis=0)
    for p_, out in zip(parts, o):
        c.add("Squeeze", [p_, c.const(np.asarray([0], np.int64))], [out])


@exporter("MergeHeads")
def _x_merge_heads(c, op, xs, i, o):
    B, H, S, D = xs[0].shape
    t = c.fresh()
    c.add("Transpose", [i[0]], [t], perm=[0, 2, 1, 3])
    c.add("Reshape", [t, c.const(np.asarray([0, 0, H * D], np.int64))], [o[0]])


@exporter("Embedding")
def _x_embedding(c, op, xs, i, o):
    c.add("Gather", [i[0], i[1]], [o[0]], axis=0)


@exporter("QKVAttention")
def _x_qkv_attention(c, op, xs, i, o):
    """Lowered as split-heads -> attention -> merge-heads (standard ONNX
    ops); the importer's fusion plan maps the attention core back."""
    from types import SimpleNamespace as NS

    B, S, E = xs[0].shape
    H = op.heads
    D = E // (3 * H)
    heads = NS(shape=(B, H, S, D))
    q, k, v, a = c.fresh(), c.fresh(), c.fresh(), c.fresh()
    _x_split_heads(c, NS(h=H), xs[:1], i[:1], [q, k, v])
    _x_attention(c, NS(scale=op.scale), [heads, heads, heads] + list(xs[1:]), [q, k, v] + list(i[1:]), [a])
    _x_merge_heads(c, None, [heads], [a], o)


@exporter("TorchCLS")
def _x_cls(c, op, xs, i, o):
    c.add("Gather", [i[0], c.const(np.asarray(0, np.int64))], [o[0]], axis=1)


def _x_spec(c, op, xs, i, o):
    """Glue operators (autograd.Fn / _Math) carry their ONNX spec."""
    spec = getattr(op, "onnx", None)
    if spec is None:
        raise NotImplementedError(f"sonnx: operator {type(op).__name__} has no ONNX lowering")
    ins = []
    for kind, v in spec["inputs"]:
        ins.append(i[v] if kind == "in" else c.const(np.asarray(v)))
    c.add(spec["op"], ins, list(o), **spec["attrs"])


def to_onnx(m, inputs: Sequence[Tensor], outputs: Optional[Sequence[Tensor]] = None, name: str = "singa_amd",
            dynamic_batch: bool = False, **fwd_kwargs):
    """Export ``m`` (a :class:`singa_amd.model.Model` or any callable taking
    ``inputs``) to an ONNX ModelProto by tracing one inference forward.
    (SINGA's ``sonnx.to_onnx(inputs, outputs)`` form is accepted when ``m``
    is a list of input tensors and ``inputs`` the outputs.)"""
    if isinstance(m, (list, tuple)) and outputs is None:
        raise ValueError("to_onnx(inputs, outputs) needs the forward to be re-run: pass the model instead")
    pnames = {}
    if hasattr(m, "get_states"):
        for k, v in m.get_states().items():
            pnames[id(v)] = k
    prev_training = autograd.training
    autograd.training = False
    autograd._TRACE.append([])
    try:
        with torch.no_grad():
            outs = m.forward(*inputs, **fwd_kwargs) if hasattr(m, "forward") else m(*inputs, **fwd_kwargs)
    finally:
        records = autograd._TRACE.pop()
        autograd.training = prev_training
    outs = list(outs) if isinstance(outs, (list, tuple)) else [outs]
    c = _ExportCtx(pnames)
    if hasattr(m, "get_states"):
        for k, v in m.get_states().items():
            if not v.stores_grad and v.data.numel() > 0:
                c.state_by_ptr[v.data.data_ptr()] = k
    g = P.new("GraphProto")
    g.name = name
    for k, x in enumerate(inputs):
        n = f"input_{k}"
        c.names[id(x)] = n
        c.keep.append(x)
        g.input.append(_value_info(n, x.shape, _T2ONNX.get(x.dtype, P.FLOAT), dynamic_batch))
    for op, xs, ys in records:
        i = [c.name_of(x) for x in xs]
        o = []
        for y in ys:
            n = c.fresh(type(op).__name__.lower())
            c.names[id(y)] = n
            c.keep.append(y)
            o.append(n)
        fn = _EXPORTERS.get(type(op).__name__)
        if fn is None and getattr(op, "onnx", None) is not None:
            fn = _x_spec  # glue operators (autograd.Fn / _Math) carry their ONNX spec
        if fn is None:
            raise NotImplementedError(f"sonnx export: no ONNX lowering for operator {type(op).__name__}")
        fn(c, op, xs, i, o)
    for k, y in enumerate(outs):
        n = c.names.get(id(y))
        if n is None:
            raise ValueError("model output was not produced by a traced operator")
        out_name = f"output_{k}"
        c.add("Identity", [n], [out_name])
        g.output.append(_value_info(out_name, y.shape, _T2ONNX.get(y.dtype, P.FLOAT), dynamic_batch))
    g.node.extend(c.nodes)
    for n, a in c.inits.items():
        tp = numpy_to_tensorproto(a, n)
        if n in c.const_names:
            tp.doc_string = CONST_TAG
        g.initializer.append(tp)
    mp = P.new("ModelProto")
    mp.ir_version = 8
    mp.producer_name = "singa_amd"
    mp.producer_version = "0.1"
    mp.graph.CopyFrom(g)
    ops = mp.opset_import.add()
    ops.domain, ops.version = "", OPSET
    return mp


def export(m, inputs, path: str, **kw) -> None:
    P.save_model(to_onnx(m, inputs, **kw), path)


# ================================================================== import
_IMPORTERS = {}


def importer(*names):
    def deco(fn):
        for n in names:
            _IMPORTERS[n] = fn
        return fn
    return deco


def _np(t) -> np.ndarray:
    if isinstance(t, Tensor):
        h = getattr(t, "_host_np", None)  # constant initializers keep their host copy: no device sync
        return h if h is not None else t.data.detach().cpu().numpy()  # (a sync cannot be captured)
    return np.asarray(t)


def _ints(t) -> List[int]:
    return [int(v) for v in _np(t).reshape(-1).tolist()]


_UNARY_IMPORT = {"Relu": autograd.relu, "Sigmoid": autograd.sigmoid, "Tanh": autograd.tanh, "Exp": autograd.exp,
                 "Log": autograd.log, "Abs": autograd.abs, "Sqrt": autograd.sqrt, "Reciprocal": autograd.reciprocal,
                 "Neg": autograd.negative, "Sign": autograd.sign, "Softplus": autograd.softplus,
                 "Softsign": autograd.softsign, "Erf": autograd.erf, "Cos": autograd.cos, "Sin": autograd.sin,
                 "Tan": autograd.tan, "Cosh": autograd.cosh, "Sinh": autograd.sinh, "Acos": autograd.acos,
                 "Asin": autograd.asin, "Atan": autograd.atan, "Acosh": autograd.acosh, "Asinh": autograd.asinh,
                 "Atanh": autograd.atanh, "Ceil": autograd.ceil, "Floor": autograd.floor, "Round": autograd.round,
                 "Identity": autograd.identity, "Selu": autograd.selu}


def _imp_unary(rep, n, x, a):
    return [_UNARY_IMPORT[n.op_type](x[0])]


for _k in _UNARY_IMPORT:
    _IMPORTERS[_k] = _imp_unary


@importer("Dropout")
def _i_dropout(rep, n, x, a):
    r = float(a.get("ratio", 0.5))
    if len(x) > 1 and x[1] is not None:
        r = float(_np(x[1]).reshape(-1)[0])
    y = autograd.dropout(x[0], r) if autograd.training and r > 0 else x[0]
    return [y] + ([None] if len(n.output) > 1 else [])


@importer("LeakyRelu")
def _i_leaky(rep, n, x, a):
    return [autograd.leakyrelu(x[0], float(a.get("alpha", 0.01)))]


@importer("Elu")
def _i_elu(rep, n, x, a):
    return [autograd.elu(x[0], float(a.get("alpha", 1.0)))]


@importer("HardSigmoid")
def _i_hsig(rep, n, x, a):
    return [autograd.hardsigmoid(x[0], float(a.get("alpha", 0.2)), float(a.get("beta", 0.5)))]


@importer("PRelu")
def _i_prelu(rep, n, x, a):
    return [autograd.prelu(x[0], x[1])]


@importer("Gelu")
def _i_gelu(rep, n, x, a):
    return [autograd.gelu(x[0])]


@importer("Add", "Sub", "Mul", "Div", "Pow")
def _i_binary(rep, n, x, a):
    f = {"Add": autograd.add, "Sub": autograd.sub, "Mul": autograd.mul, "Div": autograd.div,
         "Pow": autograd.pow}[n.op_type]
    return [f(x[0], x[1])]


@importer("MatMul")
def _i_matmul(rep, n, x, a):
    return [autograd.matmul(x[0], x[1])]


@importer("Gemm")
def _i_gemm(rep, n, x, a):
    return [autograd.gemm(x[0], x[1], x[2] if len(x) > 2 else None, float(a.get("alpha", 1.0)),
                          float(a.get("beta", 1.0)), int(a.get("transA", 0)), int(a.get("transB", 0)))]


def _conv_pads(a, nd=2):
    pads = a.get("pads", [0] * (2 * nd))
    if pads[:nd] != pads[nd:]:
        raise NotImplementedError(f"asymmetric pads {pads}")
    return tuple(pads[:nd])


@importer("Conv")
def _i_conv(rep, n, x, a):
    W = x[1]
    k = tuple(a.get("kernel_shape", W.shape[2:]))
    auto = a.get("auto_pad", "NOTSET")
    dil = tuple(a.get("dilations", [1, 1]))
    if auto in ("SAME_UPPER", "SAME_LOWER"):
        pads = ((k[0] - 1) // 2 * dil[0], (k[1] - 1) // 2 * dil[1])
    else:
        pads = _conv_pads(a)
    op = autograd.Conv2d(tuple(a.get("strides", [1, 1])), pads, dil, int(a.get("group", 1)), has_bias=len(x) > 2)
    return [op(x[0], x[1], x[2]) if len(x) > 2 else op(x[0], x[1])]


@importer("BatchNormalization")
def _i_bn(rep, n, x, a):
    rm, rv = x[3].data, x[4].data
    mom = 1.0 - float(a.get("momentum", 0.9))
    op = autograd.BatchNorm2d(rm, rv, mom, float(a.get("epsilon", 1e-5)))
    return [op(x[0], x[1], x[2])]


@importer("MaxPool", "AveragePool")
def _i_pool(rep, n, x, a):
    k = tuple(a["kernel_shape"])
    op = autograd.Pooling2d(k, tuple(a.get("strides", k)), _conv_pads(a), n.op_type == "MaxPool",
                            bool(a.get("count_include_pad", 0)), bool(a.get("ceil_mode", 0)))
    return [op(x[0])]


@importer("GlobalAveragePool")
def _i_gap(rep, n, x, a):
    return [autograd.GlobalAveragePool(True)(x[0])]


@importer("LRN")
def _i_lrn(rep, n, x, a):
    return [autograd.LRN(int(a["size"]), float(a.get("alpha", 1e-4)), float(a.get("beta", 0.75)),
                         float(a.get("bias", 1.0)))(x[0])]


@importer("Softmax")
def _i_softmax(rep, n, x, a):
    return [autograd.softmax(x[0], int(a.get("axis", -1)))]


@importer("LayerNormalization")
def _i_ln(rep, n, x, a):
    if int(a.get("axis", -1)) not in (-1, len(x[0].shape) - 1):
        raise NotImplementedError("LayerNormalization over more than the last axis")
    return [autograd.layer_norm(x[0], x[1], x[2], float(a.get("epsilon", 1e-5)))]


@importer("Reshape")
def _i_reshape(rep, n, x, a):
    shape = _ints(x[1])
    shape = [x[0].shape[i] if (d == 0 and not a.get("allowzero", 0)) else d for i, d in enumerate(shape)]
    return [autograd.reshape(x[0], shape)]


@importer("Flatten")
def _i_flatten(rep, n, x, a):
    return [autograd.flatten(x[0], int(a.get("axis", 1)))]


@importer("Transpose")
def _i_transpose(rep, n, x, a):
    return [autograd.transpose(x[0], a.get("perm"))]


@importer("Concat")
def _i_concat(rep, n, x, a):
    return [autograd.cat(list(x), int(a["axis"]))]


@importer("Split")
def _i_split(rep, n, x, a):
    ax = int(a.get("axis", 0))
    if len(x) > 1 and x[1] is not None:
        parts = _ints(x[1])
    elif "split" in a:
        parts = list(a["split"])
    else:
        k = len(n.output)
        parts = [x[0].shape[ax] // k] * k
    r = autograd.split(x[0], ax, parts)
    return list(r) if isinstance(r, tuple) else [r]


@importer("Slice")
def _i_slice(rep, n, x, a):
    st, en = _ints(x[1]), _ints(x[2])
    axes = _ints(x[3]) if len(x) > 3 and x[3] is not None else None
    steps = _ints(x[4]) if len(x) > 4 and x[4] is not None else None
    return [autograd.slice(x[0], st, en, axes, steps)]


@importer("Gather")
def _i_gather(rep, n, x, a):
    ax = int(a.get("axis", 0))
    idx = x[1]
    if ax == 0 and isinstance(idx, Tensor) and idx.creator is None and not rep.is_const(n.input[1]):
        return [autograd.embedding(idx, x[0])]
    if (ax == 0 and isinstance(idx, Tensor) and x[0].data.dim() == 2 and not idx.data.is_floating_point()
            and (_np(idx) >= 0).all()):  # constant row ids (BERT position ids): the capture-safe embedding op
        return [autograd.embedding(idx, x[0])]
    # a device-resident index (constant initializer): no host->device copy, which a HIP graph cannot capture
    return [autograd.gather(x[0], ax, idx.data if isinstance(idx, Tensor) and idx.data.device == x[0].data.device
                            else _np(idx))]


@importer("Squeeze")
def _i_squeeze(rep, n, x, a):
    ax = _ints(x[1]) if len(x) > 1 and x[1] is not None else a.get("axes")
    return [autograd.squeeze(x[0], ax)]


@importer("Unsqueeze")
def _i_unsqueeze(rep, n, x, a):
    ax = _ints(x[1]) if len(x) > 1 and x[1] is not None else a.get("axes")
    return [autograd.unsqueeze(x[0], ax)]


@importer("ReduceMean", "ReduceSum")
def _i_reduce(rep, n, x, a):
    ax = _ints(x[1]) if len(x) > 1 and x[1] is not None else a.get("axes")
    kd = int(a.get("keepdims", 1))
    f = autograd.reduce_mean if n.op_type == "ReduceMean" else autograd.reduce_sum
    return [f(x[0], ax, kd)]


@importer("Cast")
def _i_cast(rep, n, x, a):
    to = int(a["to"])
    dt = {P.FLOAT: torch.float32, P.INT64: torch.int64, P.INT32: torch.int32, P.BOOL: torch.bool,
          P.FLOAT16: torch.float16, P.DOUBLE: torch.float32, P.UINT8: torch.uint8}[to]
    if x[0].creator is None or not dt.is_floating_point:
        return [Tensor(device=x[0].device, data=x[0].data.to(dt), requires_grad=False)]
    return [autograd.cast(x[0], dt)]


@importer("Constant")
def _i_constant(rep, n, x, a):
    v = a.get("value")
    if v is None:
        v = np.asarray(a.get("value_float", a.get("value_int", 0)))
    return [rep.const_tensor(np.asarray(v))]


@importer("Shape")
def _i_shape(rep, n, x, a):
    return [rep.const_tensor(np.asarray(x[0].shape, np.int64))]


@importer("ConstantOfShape")
def _i_cos(rep, n, x, a):
    v = a.get("value")
    val = float(np.asarray(v).reshape(-1)[0]) if v is not None else 0.0
    dt = np.asarray(v).dtype if v is not None else np.float32
    return [rep.const_tensor(np.full(_ints(x[0]), val, dtype=dt))]


@importer("Where")
def _i_where(rep, n, x, a):
    return [autograd.where(x[1], x[2], x[0])]


@importer("Equal", "Less", "Greater", "And", "Or", "Xor")
def _i_cmp(rep, n, x, a):
    f = {"Equal": autograd.equal, "Less": autograd.less, "Greater": autograd.greater, "And": autograd._and,
         "Or": autograd._or, "Xor": autograd._xor}[n.op_type]
    return [f(x[0], x[1])]


@importer("Not")
def _i_not(rep, n, x, a):
    return [autograd._not(x[0])]


@importer("Clip")
def _i_clip(rep, n, x, a):
    lo = float(_np(x[1]).reshape(-1)[0]) if len(x) > 1 and x[1] is not None else a.get("min")
    hi = float(_np(x[2]).reshape(-1)[0]) if len(x) > 2 and x[2] is not None else a.get("max")
    return [autograd.clip(x[0], lo, hi)]


@importer("Pad")
def _i_pad(rep, n, x, a):
    pads = _ints(x[1]) if len(x) > 1 else a.get("pads")
    cval = float(_np(x[2]).reshape(-1)[0]) if len(x) > 2 and x[2] is not None else 0.0
    return [autograd.pad(x[0], a.get("mode", "constant"), pads, cval)]


@importer("Expand")
def _i_expand(rep, n, x, a):
    shp = _ints(x[1])
    out = list(np.broadcast_shapes(tuple(x[0].shape), tuple(shp)))
    return [autograd.expand(x[0], out)]


@importer("Tile")
def _i_tile(rep, n, x, a):
    return [autograd.tile(x[0], _ints(x[1]))]


@importer("Min", "Max", "Sum", "Mean")
def _i_variadic(rep, n, x, a):
    f = {"Min": autograd.min, "Max": autograd.max, "Sum": autograd.sum, "Mean": autograd.mean}[n.op_type]
    return [f(*x)]


@importer("Resize", "Upsample")
def _i_resize(rep, n, x, a):
    sc = x[2] if n.op_type == "Resize" else x[1]
    return [autograd.upsample(x[0], "nearest", _np(sc).reshape(-1).tolist())]


@importer("DepthToSpace")
def _i_d2s(rep, n, x, a):
    return [autograd.depth_to_space(x[0], int(a["blocksize"]), a.get("mode", "DCR"))]


@importer("SpaceToDepth")
def _i_s2d(rep, n, x, a):
    return [autograd.space_to_depth(x[0], int(a["blocksize"]))]


@importer("ScatterElements")
def _i_scatter(rep, n, x, a):
    return [autograd.scatter_elements(x[0], x[1], x[2], int(a.get("axis", 0)))]


@importer("OneHot")
def _i_onehot(rep, n, x, a):
    return [autograd.onehot(int(a.get("axis", -1)), x[0], int(_np(x[1]).reshape(-1)[0]), x[2])]


# ------------------------------------------------------ import-time fusion
class _Fused:
    """One fused group of imported nodes: runs at the position of its LAST
    member (every external input exists by then) and defines only the
    group's final output (the intermediates have no other consumer)."""

    def __init__(self, kind: str, members, inputs, output: str, scale: Optional[float] = None, heads: int = 0):
        self.kind, self.members, self.inputs, self.output, self.scale = kind, tuple(members), list(inputs), output, scale
        self.heads = heads

    def _low(self, rep, t):
        cd = rep.compute_dtype
        return autograd.cast(t, cd) if cd is not None and t.data.is_cuda and t.dtype == torch.float32 else t

    def run(self, rep, xs):
        if self.kind == "linear":  # MatMul + bias Add -> one GEMM with a bias epilogue (bf16 weight copy)
            return autograd.linear(self._low(rep, xs[0]), xs[1], xs[2])
        if self.kind == "gelu":  # x * 0.5 * (1 + erf(x / sqrt 2)) -> one elementwise kernel
            return autograd.gelu(xs[0])
        if self.kind == "linear_gelu":  # MatMul + bias Add + GELU chain -> one GEMM, GELU in its epilogue
            return autograd.linear(self._low(rep, xs[0]), xs[1], xs[2], act="gelu")
        if self.kind == "qkv_attention":  # split-heads + attention + merge-heads -> heads addressed in place
            att = autograd.QKVAttention(self.heads, self.scale)
            qkv = self._low(rep, xs[0])
            return att(qkv, xs[1]) if len(xs) > 1 else att(qkv)
        if self.kind == "attention":  # Transpose/MatMul/scale/[mask]/Softmax/MatMul -> batched-MFMA attention
            q, k, v = (self._low(rep, t) for t in xs[:3])
            return autograd.attention(q, k, v, xs[3] if len(xs) > 3 else None, self.scale)
        if self.kind == "add_ln":  # [Identity] + Add + LayerNormalization -> one residual-tail operator
            x, a, g, b = xs
            if x.data.is_cuda and x.dtype != a.dtype and {x.dtype, a.dtype} == {torch.float32, torch.bfloat16}:
                # mixed-precision import: the residual stream joins the compute
                # dtype here (once, after the fp32 embedding LayerNorm), as in
                # the native bf16 model -- every later projection input is then
                # already bf16 (no per-GEMM input casts), the tail runs on bf16
                # bytes and its input a is the projection's own output (so the
                # tail can sum that projection's bias gradient in place)
                lo = rep.compute_dtype if rep.compute_dtype in (torch.float32, torch.bfloat16) else torch.float32
                x, a = (autograd.cast(x, lo) if x.dtype != lo else x), (autograd.cast(a, lo) if a.dtype != lo else a)
            if not autograd._TRACE and x.data.is_cuda and F.drop_add_ln_ok(x.data, a.data):
                return autograd.DropAddLayerNorm(0.0, None, self.scale)(x, a, g, b)
            return autograd.layer_norm(autograd.add(x, a), g, b, self.scale)
        raise ValueError(self.kind)

    def __repr__(self):
        return f"_Fused({self.kind}, nodes={list(self.members)}, out={self.output!r})"


# doc_string of an exported initializer that is a constant (GELU's sqrt 2, the
# attention scale, BN running statistics, ...) rather than a parameter: ONNX
# itself does not say which initializers are trainable
CONST_TAG = "singa_amd:const"


def _fusion_plan(nodes, inits: Dict[str, Tensor], consts: set, outputs: Sequence[str],
                 gelu_scalars: Optional[set] = None) -> Dict[int, _Fused]:
    """Pattern-match the imported node list into fused groups, keyed by the
    index of each group's last node:

    * ``linear``    MatMul(x, W) -> Add(., b), W [in, out] and b [out] parameters;
    * ``gelu``      Div(x, sqrt 2) -> Erf -> Add(., 1) -> Mul(x, .) -> Mul(., 0.5)
                    (the exact-erf GELU both this exporter and PyTorch's emit);
    * ``attention`` Transpose(k, swap last two) -> MatMul(q, .) -> Mul/Div(., c)
                    -> [Add(., mask)] -> Softmax(last axis) -> MatMul(., v).

    A chain only fuses when every intermediate has exactly one consumer and
    is not a graph output, so no other node can observe what it skips.  The
    unfused import runs 2 / 5 / 5-6 autograd ops (and their backward kernels)
    per group, plus an fp32->bf16 cast of every MatMul weight per step.

    A ``linear`` whose output only feeds a ``gelu`` becomes one
    ``linear_gelu`` (the GELU runs in the GEMM epilogue).

    ``gelu_scalars``: untagged one-element initializers the GELU pattern may
    consume as its constants (sqrt 2, 1, 0.5 -- values checked exactly); the
    importer freezes the ones a matched GELU used.  Every other pattern
    constant must be a tagged constant, so a learnable scalar (a temperature
    feeding the attention scores) keeps its gradient and blocks the fusion."""
    cons: Dict[str, List[int]] = {}
    soft = gelu_scalars or set()
    for idx, nd in enumerate(nodes):
        for nm in nd.input:
            if nm:
                cons.setdefault(nm, []).append(idx)
    outs = set(outputs)
    used: set = set()

    def only(name: str) -> Optional[int]:
        c = cons.get(name, [])
        if len(c) != 1 or name in outs or c[0] in used:
            return None
        return c[0]

    def scalar(name: str, allow_soft: bool = False) -> Optional[float]:
        t = inits.get(name)
        if t is None or t.data.numel() != 1 or not (name in consts or (allow_soft and name in soft)):
            return None
        return float(t.data.reshape(-1)[0])

    def param(name: str, dim: int) -> bool:
        t = inits.get(name)
        return t is not None and t.stores_grad and t.data.dim() == dim

    def attr(nd, key, default=None):
        for a in nd.attribute:
            if a.name == key:
                return attr_value(a)
        return default

    def other(nd, name: str) -> Optional[str]:
        ins = list(nd.input)
        if len(ins) != 2 or name not in ins:
            return None
        return ins[1] if ins[0] == name else ins[0]

    def linear(i):
        nd = nodes[i]
        if nd.op_type != "MatMul" or not param(nd.input[1], 2):
            return None
        j = only(nd.output[0])
        if j is None or nodes[j].op_type != "Add":
            return None
        b = other(nodes[j], nd.output[0])
        if b is None or not param(b, 1) or inits[b].data.shape[0] != inits[nd.input[1]].data.shape[1]:
            return None
        return _Fused("linear", (i, j), [nd.input[0], nd.input[1], b], nodes[j].output[0])

    def gelu(i):
        nd = nodes[i]
        s2 = scalar(nd.input[1], True) if nd.op_type == "Div" else None
        if s2 is None or abs(s2 - math.sqrt(2.0)) > 1e-4:
            return None
        x = nd.input[0]
        j = only(nd.output[0])
        if j is None or nodes[j].op_type != "Erf":
            return None
        k = only(nodes[j].output[0])
        if k is None or nodes[k].op_type != "Add":
            return None
        c = other(nodes[k], nodes[j].output[0])
        if c is None or scalar(c, True) != 1.0:
            return None
        m = only(nodes[k].output[0])
        if m is None or nodes[m].op_type != "Mul" or other(nodes[m], nodes[k].output[0]) != x:
            return None
        n = only(nodes[m].output[0])
        if n is None or nodes[n].op_type != "Mul":
            return None
        h = other(nodes[n], nodes[m].output[0])
        if h is None or scalar(h, True) != 0.5:
            return None
        return _Fused("gelu", (i, j, k, m, n), [x], nodes[n].output[0])

    def attention(i):
        nd = nodes[i]
        perm = attr(nd, "perm")
        if nd.op_type != "Transpose" or not perm or len(perm) < 2:
            return None
        r = len(perm)
        if list(perm) != list(range(r - 2)) + [r - 1, r - 2]:
            return None
        j = only(nd.output[0])
        if j is None or nodes[j].op_type != "MatMul" or nodes[j].input[1] != nd.output[0]:
            return None
        q, k_ = nodes[j].input[0], nd.input[0]
        m = only(nodes[j].output[0])
        if m is None or nodes[m].op_type not in ("Mul", "Div"):
            return None
        c = scalar(nodes[m].input[1]) if nodes[m].input[0] == nodes[j].output[0] else None
        if c is None and nodes[m].op_type == "Mul":
            c = scalar(nodes[m].input[0]) if nodes[m].input[1] == nodes[j].output[0] else None
        if c is None or c == 0.0:
            return None
        scale = c if nodes[m].op_type == "Mul" else 1.0 / c
        members, cur, mask = [i, j, m], nodes[m].output[0], None
        s = only(cur)
        if s is not None and nodes[s].op_type == "Add":
            mask = other(nodes[s], cur)
            if mask is None or mask in inits and inits[mask].stores_grad:
                return None
            members.append(s)
            cur = nodes[s].output[0]
            s = only(cur)
        if s is None or nodes[s].op_type != "Softmax" or int(attr(nodes[s], "axis", -1)) not in (-1, r - 1):
            return None
        members.append(s)
        t = only(nodes[s].output[0])
        if t is None or nodes[t].op_type != "MatMul" or nodes[t].input[0] != nodes[s].output[0]:
            return None
        members.append(t)
        ins = [q, k_, nodes[t].input[1]] + ([mask] if mask is not None else [])
        return _Fused("attention", members, ins, nodes[t].output[0], scale)

    prod = {o: idx for idx, nd in enumerate(nodes) for o in nd.output if o}

    def single(name: str) -> bool:  # exactly one consumer, not a graph output
        return len(cons.get(name, [])) == 1 and name not in outs

    def host_ints(name: str):
        t = inits.get(name)
        h = getattr(t, "_host_np", None) if t is not None else None
        return None if h is None else [int(v) for v in np.asarray(h).reshape(-1)]

    def qkv_heads(st):
        """Extend an attention group over the split-heads chain in front of
        it -- Reshape([0,0,3,H,D]) -> Transpose([2,0,3,1,4]) -> Split(axis 0)
        -> Squeeze x3 -- and the merge-heads chain behind it -- Transpose
        ([0,2,1,3]) -> Reshape([0,0,H*D])."""
        q, k_, v = st.inputs[:3]
        sq = [prod.get(t) for t in (q, k_, v)]
        if any(j is None or nodes[j].op_type != "Squeeze" or j in used or not single(t) for j, t in zip(sq, (q, k_, v))):
            return None
        srcs = [nodes[j].input[0] for j in sq]
        sp = prod.get(srcs[0])
        if sp is None or sp in used or nodes[sp].op_type != "Split" or list(nodes[sp].output) != srcs:
            return None
        if int(attr(nodes[sp], "axis", 0)) != 0 or not all(single(t) for t in srcs):
            return None
        t5 = nodes[sp].input[0]
        tr = prod.get(t5)
        if tr is None or tr in used or nodes[tr].op_type != "Transpose" or not single(t5):
            return None
        if list(attr(nodes[tr], "perm", [])) != [2, 0, 3, 1, 4]:
            return None
        r5 = nodes[tr].input[0]
        rs = prod.get(r5)
        if rs is None or rs in used or nodes[rs].op_type != "Reshape" or not single(r5):
            return None
        shp = host_ints(nodes[rs].input[1])
        if shp is None or len(shp) != 5 or shp[2] != 3 or shp[0] != 0 or shp[1] != 0:
            return None
        H, D = shp[3], shp[4]
        a = st.output
        if not single(a):
            return None
        t2 = cons[a][0]
        if t2 in used or nodes[t2].op_type != "Transpose" or list(attr(nodes[t2], "perm", [])) != [0, 2, 1, 3]:
            return None
        if not single(nodes[t2].output[0]):
            return None
        r2 = cons[nodes[t2].output[0]][0]
        if r2 in used or nodes[r2].op_type != "Reshape" or host_ints(nodes[r2].input[1]) != [0, 0, H * D]:
            return None
        members = list(st.members) + sq + [sp, tr, rs, t2, r2]
        return _Fused("qkv_attention", members, [nodes[rs].input[0]] + st.inputs[3:], nodes[r2].output[0], st.scale,
                      heads=H)

    plan: Dict[int, _Fused] = {}
    for i in range(len(nodes)):
        if i in used:
            continue
        for pat in (attention, gelu, linear):
            st = pat(i)
            if st is not None:
                used.update(st.members)
                plan[max(st.members)] = st
                break
    for key, st in list(plan.items()):
        if st.kind == "attention":
            big = qkv_heads(st)
            if big is not None:
                del plan[key]
                used.update(big.members)
                plan[max(big.members)] = big
    # residual tails: [Identity (an exported dropout)] -> Add(x, a) ->
    # LayerNormalization(last axis) -> one DropAddLayerNorm (one pass each
    # way; the Linear producing a gets its bias gradient from the tail's
    # backward): the operand a Linear group produces goes second
    lin_outs = {st.output for st in plan.values() if st.kind in ("linear", "linear_gelu")}
    for i, nd in enumerate(nodes):
        if i in used or nd.op_type != "Add" or len(nd.input) != 2:
            continue
        j = only(nd.output[0])
        if j is None or nodes[j].op_type != "LayerNormalization" or len(nodes[j].input) != 3:
            continue
        ax = int(attr(nodes[j], "axis", -1))
        if ax != -1:
            continue
        members, ops = [i, j], []
        for t in nd.input:
            p = prod.get(t)
            if p is not None and p not in used and nodes[p].op_type == "Identity" and single(t):
                members.append(p)
                t = nodes[p].input[0]
            ops.append(t)
        if ops[0] in lin_outs and ops[1] not in lin_outs:
            ops.reverse()
        used.update(members)
        plan[max(members)] = _Fused("add_ln", members, ops + list(nodes[j].input[1:3]), nodes[j].output[0],
                                    float(attr(nodes[j], "epsilon", 1e-5)))
    # a Linear whose output feeds only a GELU chain -> one GEMM with the GELU
    # in its epilogue (and its derivative in the consumer's data gradient)
    lin_by_out = ({st.output: k for k, st in plan.items() if st.kind == "linear"}
                  if os.environ.get("SINGA_AMD_FUSE_GELU", "0") != "0" else {})
    for key, st in list(plan.items()):
        if st.kind != "gelu":
            continue
        x = st.inputs[0]
        lk = lin_by_out.get(x)
        if lk is None or x in outs or not set(cons.get(x, [])) <= set(st.members):
            continue
        lin = plan.pop(lk)
        del plan[key]
        plan[max(st.members)] = _Fused("linear_gelu", tuple(lin.members) + tuple(st.members), lin.inputs, st.output)
    return plan


class SingaRep:
    """An imported ONNX graph bound to a device (SINGA ``SingaRep``).

    Import-time fusion (``fuse=True``, default; ``SINGA_AMD_SONNX_FUSE=0``
    turns it off) maps the exported Linear / GELU / attention node chains
    back onto the fused autograd operators (:func:`_fusion_plan`)."""

    # ops whose float operands run at ``compute_dtype`` (MFMA GEMM / conv);
    # everything else (softmax, norms, elementwise) sees what they produce
    _LOWP = {"MatMul": (0, 1), "Gemm": (0, 1), "Conv": (0, 1), "ConvTranspose": (0, 1)}

    def __init__(self, mp, device=None, trainable: bool = True, compute_dtype=None, fuse: Optional[bool] = None):
        from .. import device as _dev

        self.model_proto = mp
        # autocast-style mixed precision for imported graphs (fp32 master
        # weights; GEMM-shaped ops cast their operands, grads flow back in fp32)
        self.compute_dtype = compute_dtype
        self.device = device or _dev.get_default_device()
        g = mp.graph
        self.graph = g
        self.inits: Dict[str, Tensor] = OrderedDict()
        self._consts = set()
        weight_like = self._weight_inputs(g)
        consumers: Dict[str, set] = {}
        for nd in g.node:
            for nm in nd.input:
                consumers.setdefault(nm, set()).add(nd.op_type)
        scalar_math = {"Add", "Mul", "Sub", "Div", "Pow"}
        soft, soft_np = set(), {}
        for t in g.initializer:
            a = tensorproto_to_numpy(t)
            # constants are what the exporter tagged as such; an untagged
            # initializer in a learnable position is a parameter, scalars
            # included (a learnable temperature / scale) -- except the GELU
            # pattern's numeric constants, frozen below when the pattern matches
            tagged = t.doc_string == CONST_TAG
            is_param = trainable and a.dtype == np.float32 and t.name in weight_like and not tagged
            if is_param and a.size == 1 and consumers.get(t.name, set()) <= scalar_math:
                soft.add(t.name)
                soft_np[t.name] = a
            ten = Tensor(device=self.device, data=torch.from_numpy(np.array(a, order="C")),
                         requires_grad=is_param, stores_grad=is_param)
            ten.name = t.name
            if not is_param:
                self._consts.add(t.name)
                ten._host_np = a
            self.inits[t.name] = ten
        init_names = set(self.inits)
        self.input_names = [v.name for v in g.input if v.name not in init_names]
        self.output_names = [v.name for v in g.output]
        for nd in g.node:
            if nd.op_type not in _IMPORTERS:
                raise NotImplementedError(f"sonnx import: unsupported ONNX op {nd.op_type}")
        if fuse is None:
            fuse = os.environ.get("SINGA_AMD_SONNX_FUSE", "1") != "0"
        self.fused = _fusion_plan(list(g.node), self.inits, self._consts, self.output_names, soft) if fuse else {}
        for st in self.fused.values():
            if st.kind not in ("gelu", "linear_gelu"):
                continue
            for i in st.members:
                for nm in g.node[i].input:
                    if nm in soft and nm not in self._consts:  # a matched GELU's constant: freeze it
                        ten = self.inits[nm]
                        ten.requires_grad = ten.stores_grad = False
                        ten._host_np = soft_np[nm]
                        self._consts.add(nm)
        self._skip = {i for st in self.fused.values() for i in st.members}

    @staticmethod
    def _weight_inputs(g) -> set:
        """Initializer names consumed in a learnable position."""
        pos = {"Conv": (1, 2), "Gemm": (1, 2), "MatMul": (0, 1), "BatchNormalization": (1, 2),
               "LayerNormalization": (1, 2), "Add": (0, 1), "Mul": (0, 1), "Sub": (0, 1), "Gather": (0,),
               "PRelu": (1,)}
        out = set()
        for nd in g.node:
            for k in pos.get(nd.op_type, ()):
                if k < len(nd.input):
                    out.add(nd.input[k])
        return out

    def is_const(self, name: str) -> bool:
        return name in self._consts

    def const_tensor(self, a: np.ndarray) -> Tensor:
        t = Tensor(device=self.device, data=torch.from_numpy(np.array(a, order="C")), requires_grad=False)
        t._host_np = np.asarray(a)
        return t

    def params(self) -> Dict[str, Tensor]:
        return OrderedDict((k, v) for k, v in self.inits.items() if v.stores_grad)

    def run(self, inputs: Sequence, **kw) -> List[Tensor]:
        env: Dict[str, Optional[Tensor]] = dict(self.inits)
        for name, x in zip(self.input_names, inputs):
            if not isinstance(x, Tensor):
                x = Tensor(device=self.device, data=torch.as_tensor(np.asarray(x)), requires_grad=False)
            env[name] = x
        for idx, nd in enumerate(self.graph.node):
            st = self.fused.get(idx)
            if st is not None:
                env[st.output] = st.run(self, [env.get(i) if i else None for i in st.inputs])
                continue
            if idx in self._skip:
                continue
            attrs = {a.name: attr_value(a) for a in nd.attribute}
            xs = [env.get(i) if i else None for i in nd.input]
            if self.compute_dtype is not None and nd.op_type in self._LOWP:
                for k in self._LOWP[nd.op_type]:
                    if k < len(xs) and xs[k] is not None and xs[k].dtype == torch.float32:
                        xs[k] = autograd.cast(xs[k], self.compute_dtype)
            ys = _IMPORTERS[nd.op_type](self, nd, xs, attrs)
            for name, y in zip(nd.output, ys):
                if name:
                    env[name] = y
        return [env[n] for n in self.output_names]


class SingaBackend:
    """``sonnx.SingaBackend.prepare(model, device)`` / ``run_model``."""

    @staticmethod
    def prepare(mp, device=None, **kw) -> SingaRep:
        if isinstance(mp, (str, bytes, bytearray)):
            mp = P.load_model(mp)
        return SingaRep(mp, device, **kw)

    @staticmethod
    def run_model(mp, inputs, device=None):
        return SingaBackend.prepare(mp, device).run(inputs)


prepare = SingaBackend.prepare
run_model = SingaBackend.run_model
backend = SingaBackend


class SONNXModel(model.Model):
    """A trainable model built from an ONNX graph (SINGA ``sonnx.SONNXModel``):
    ``forward(*inputs)`` runs the graph; initializers in weight positions are
    parameters the optimiser updates (fine-tuning)."""

    def __init__(self, onnx_model, device=None, loss=None, compute_dtype=None):
        super().__init__()
        self.rep = prepare(onnx_model, device, compute_dtype=compute_dtype)
        if compute_dtype is not None:  # fp32 master weights + the optimiser's bf16 compute copies (fused Linear)
            self.compute_dtype = compute_dtype
        self._onnx_params = self.rep.params()
        for k, v in self._onnx_params.items():
            v.param_meta = {"lr_mult": 1.0, "wd_mult": 1.0}
        from .. import layer

        self.loss_fn = loss or layer.SoftMaxCrossEntropy()

    def get_params(self, prefix: str = "") -> Dict[str, Tensor]:
        return OrderedDict((prefix + k, v) for k, v in self._onnx_params.items())

    def get_states(self, prefix: str = "") -> Dict[str, Tensor]:
        return OrderedDict((prefix + k, v) for k, v in self.rep.inits.items())

    def forward(self, *xs):
        outs = self.rep.run(xs)
        return outs[0] if len(outs) == 1 else outs

    def train_one_batch(self, x, y, *extra):
        out = self.forward(x, *extra)
        loss = self.loss_fn(out, y)
        self.optimizer(loss)
        return out, loss


__all__ = ["to_onnx", "export", "prepare", "run_model", "SingaBackend", "SingaRep", "SONNXModel", "make_node",
           "make_attribute", "numpy_to_tensorproto", "tensorproto_to_numpy", "OPSET"]
