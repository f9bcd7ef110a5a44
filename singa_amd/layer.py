"""``singa_amd.layer`` -- SINGA's stateful layer API (lazy parameter init).

Layers create their parameters on the first call, when the input shape is
known (like SINGA's ``Layer.initialize``).  Parameter tensors have
``stores_grad=True``; :class:`singa_amd.opt.ParamStore` later re-homes them
into one flat fp32 buffer (+ bf16 compute copy).  Initialisers follow the
reference's ParamProto init methods (src/utils/param.cc:89-127); the
InnerProduct fan-in bug (fan_in = in*out) is not
reproduced.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import autograd
from .ops import glue as G
from . import device as _dev
from .tensor import Tensor


def _pair(v) -> Tuple[int, int]:
    if isinstance(v, (list, tuple)):
        return (int(v[0]), int(v[1]))
    return (int(v), int(v))


class Layer:
    sep = "."

    def __init__(self):
        self.name = None
        self._initialized = False
        self._params: "OrderedDict[str, Tensor]" = OrderedDict()
        self._states: "OrderedDict[str, Tensor]" = OrderedDict()
        self._layers: "OrderedDict[str, Layer]" = OrderedDict()

    # attribute registration (sub-layers / params) --------------------------
    def __setattr__(self, key, value):
        if isinstance(value, Layer):
            self.__dict__.setdefault("_layers", OrderedDict())[key] = value
            if value.name is None:
                value.name = key
        elif (isinstance(value, (list, tuple)) and any(isinstance(v, Layer) for v in value)
              and all(isinstance(v, Layer) or v is None for v in value)):
            d = self.__dict__.setdefault("_layers", OrderedDict())
            for i, v in enumerate(value):
                if v is None:
                    continue
                d[f"{key}.{i}"] = v
                if v.name is None:
                    v.name = f"{key}.{i}"
        super().__setattr__(key, value)

    def _sublayers(self) -> "OrderedDict[str, Layer]":
        """Direct sub-layers in attribute order, re-scanned on every call so a
        list filled AFTER its assignment (``self.blocks = []`` then
        ``append``) is still found."""
        out = OrderedDict()
        for key, v in self.__dict__.items():
            if key.startswith("_"):
                continue
            if isinstance(v, Layer):
                out[key] = v
            elif isinstance(v, (list, tuple)) and v and all(isinstance(e, Layer) or e is None for e in v):
                for i, e in enumerate(v):
                    if e is not None:
                        if e.name is None:
                            e.name = f"{key}.{i}"
                        out[f"{key}.{i}"] = e
        return out

    def _param(self, key: str, t: Tensor, lr_mult: float = 1.0, wd_mult: float = 1.0) -> Tensor:
        t.stores_grad = True
        t.requires_grad = True
        t.name = key
        t.param_meta = {"lr_mult": lr_mult, "wd_mult": wd_mult}
        self._params[key] = t
        setattr(self, key, t)
        return t

    def _state(self, key: str, t: Tensor) -> Tensor:
        t.requires_grad = False
        t.stores_grad = False
        self._states[key] = t
        setattr(self, key, t)
        return t

    def __call__(self, *args, **kwargs):
        if not self._initialized:
            self.initialize(*args, **kwargs)
            self._initialized = True
        return self.forward(*args, **kwargs)

    def initialize(self, *args, **kwargs):
        pass

    def forward(self, *args, **kwargs):
        raise NotImplementedError

    @property
    def device(self):
        for p in self._params.values():
            return p.device
        return _dev.get_default_device()

    # params / states -----------------------------------------------------
    def get_params(self, prefix: str = "") -> Dict[str, Tensor]:
        out = OrderedDict()
        for k, v in self._params.items():
            out[prefix + k] = v
        for ln, l in self._sublayers().items():
            out.update(l.get_params(prefix + ln + self.sep))
        return out

    def _flat_params(self) -> List[Tensor]:
        seen, out = set(), []
        for p in self.get_params().values():
            if id(p) not in seen:
                seen.add(id(p))
                out.append(p)
        return out

    def get_states(self, prefix: str = "") -> Dict[str, Tensor]:
        out = OrderedDict()
        for k, v in self._params.items():
            out[prefix + k] = v
        for k, v in self._states.items():
            out[prefix + k] = v
        for ln, l in self._sublayers().items():
            out.update(l.get_states(prefix + ln + self.sep))
        return out

    @staticmethod
    def _assign(dst: Tensor, v) -> None:
        if isinstance(v, Tensor):
            src = v.data
        elif isinstance(v, torch.Tensor):
            src = v
        else:
            src = torch.as_tensor(np.asarray(v))
        G.copy_(dst.data, src.reshape(dst.shape))
        if dst.low is not None:
            G.copy_(dst.low, dst.data)

    def set_params(self, parameters: Dict[str, Tensor]) -> None:
        own = self.get_params()
        for k, v in parameters.items():
            if k in own:
                self._assign(own[k], v)

    def set_states(self, states: Dict[str, Tensor]) -> None:
        own = self.get_states()
        for k, v in states.items():
            if k in own:
                self._assign(own[k], v)

    def dtype_check(self, *inputs):
        pass


def _new_param(shape, dev, dtype=torch.float32) -> Tensor:
    return Tensor(shape, dev, dtype, requires_grad=True, stores_grad=True)


class Linear(Layer):
    """y = act(x W + b), W [in, out].  ``activation`` (relu / sigmoid / tanh /
    stanh / gelu / gelu_tanh, default none) is applied in the GEMM epilogue,
    and its backward in the next fused Linear's data-gradient epilogue (see
    autograd.Linear)."""

    def __init__(self, out_features: int, *args, bias: bool = True, activation: Optional[str] = None, **kwargs):
        super().__init__()
        self.in_features = None
        if len(args) > 0:  # Linear(in, out[, bias])
            self.in_features = out_features
            out_features = args[0]
            if len(args) > 1:
                bias = args[1]
        self.out_features = out_features
        self.bias = bias
        if activation is not None and activation not in ("relu", "sigmoid", "tanh", "stanh", "gelu", "gelu_tanh"):
            raise ValueError(f"Linear: unsupported fused activation {activation}")
        self.activation = activation

    def initialize(self, x):
        self.in_features = x.shape[-1]
        dev = x.device
        std = math.sqrt(2.0 / (self.in_features + self.out_features))
        W = _new_param((self.in_features, self.out_features), dev)
        W.gaussian(0.0, std)
        self._param("W", W)
        if self.bias:
            self._param("b", _new_param((self.out_features,), dev), wd_mult=0.0)

    def forward(self, x):
        if self.bias:
            return autograd.Linear(True, act=self.activation)(x, self.W, self.b)
        return autograd.Linear(False, act=self.activation)(x, self.W)


class Gemm(Layer):
    def __init__(self, nb_kernels, alpha=1.0, beta=1.0, transA=False, transB=True, bias=True):
        super().__init__()
        self.nb_kernels, self.alpha, self.beta, self.transA, self.transB, self.bias_ = \
            nb_kernels, alpha, beta, transA, transB, bias

    def initialize(self, x):
        k = x.shape[0] if self.transA else x.shape[1]
        shp = (self.nb_kernels, k) if self.transB else (k, self.nb_kernels)
        W = _new_param(shp, x.device)
        W.gaussian(0.0, math.sqrt(2.0 / (k + self.nb_kernels)))
        self._param("W", W)
        if self.bias_:
            self._param("b", _new_param((1, self.nb_kernels), x.device), wd_mult=0.0)

    def forward(self, x):
        return autograd.gemm(x, self.W, self.b if self.bias_ else None, self.alpha, self.beta, int(self.transA),
                             int(self.transB))


class Conv2d(Layer):
    def __init__(self, nb_kernels: int, kernel_size, *args, stride=1, padding=0, dilation=1, group=1, bias=True,
                 pad_mode="NOTSET", activation="NOTSET", **kwargs):
        super().__init__()
        self.in_channels = None
        if len(args) > 0:  # Conv2d(in, out, kernel, ...)
            self.in_channels = nb_kernels
            nb_kernels = kernel_size
            kernel_size = args[0]
        self.nb_kernels = nb_kernels
        self.kernel_size = _pair(kernel_size)
        self.stride = _pair(stride)
        self.padding = _pair(padding)
        self.dilation = _pair(dilation)
        self.group = group
        self.bias = bias
        self.pad_mode = pad_mode
        self.activation = activation

    def initialize(self, x):
        C = self.in_channels or x.shape[1]
        self.in_channels = C
        if self.pad_mode in ("SAME_UPPER", "SAME_LOWER"):
            self.padding = ((self.kernel_size[0] - 1) // 2 * self.dilation[0],
                            (self.kernel_size[1] - 1) // 2 * self.dilation[1])
        shape = (self.nb_kernels, C // self.group) + self.kernel_size
        W = _new_param(shape, x.device)
        std = math.sqrt(2.0 / (C * self.kernel_size[0] * self.kernel_size[1] + self.nb_kernels))
        W.gaussian(0.0, std)
        self._param("W", W)
        if self.bias:
            self._param("b", _new_param((self.nb_kernels,), x.device), wd_mult=0.0)

    def forward(self, x):
        op = autograd.Conv2d(self.stride, self.padding, self.dilation, self.group, has_bias=self.bias,
                             fuse_relu=(self.activation == "RELU"), bn_stats=getattr(self, "bn_stats", False))
        return op(x, self.W, self.b) if self.bias else op(x, self.W)


class SeparableConv2d(Layer):
    def __init__(self, nb_kernels, kernel_size, *args, stride=1, padding=0, bias=False):
        super().__init__()
        self.nb_kernels, self.kernel_size, self.stride, self.padding, self.bias = \
            nb_kernels, kernel_size, stride, padding, bias

    def initialize(self, x):
        C = x.shape[1]
        self.depthwise_conv = Conv2d(C, self.kernel_size, stride=self.stride, padding=self.padding, group=C,
                                     bias=self.bias)
        self.point_conv = Conv2d(self.nb_kernels, 1, bias=self.bias)

    def forward(self, x):
        return self.point_conv(self.depthwise_conv(x))


class BatchNorm2d(Layer):
    """SINGA convention: running = momentum*running + (1-momentum)*batch."""

    def __init__(self, *args, momentum: float = 0.9, eps: float = 1e-5):
        super().__init__()
        self.momentum = momentum
        self.eps = eps

    def initialize(self, x, *args, **kwargs):
        C = x.shape[1]
        dev = x.device
        s = _new_param((C,), dev)
        G.fill_(s.data, 1.0)
        self._param("scale", s, wd_mult=0.0)
        self._param("bias", _new_param((C,), dev), wd_mult=0.0)
        self._state("running_mean", Tensor((C,), dev, requires_grad=False))
        rv = Tensor((C,), dev, requires_grad=False)
        G.fill_(rv.data, 1.0)
        self._state("running_var", rv)

    def forward(self, x, relu: bool = False, residual: Optional[Tensor] = None, colsum: bool = False):
        op = autograd.BatchNorm2d(self.running_mean.data, self.running_var.data, 1.0 - self.momentum, self.eps,
                                  relu=relu, has_residual=residual is not None, colsum=colsum)
        if residual is not None:
            return op(x, self.scale, self.bias, residual)
        return op(x, self.scale, self.bias)


class LayerNorm(Layer):
    def __init__(self, eps=1e-5):
        super().__init__()
        self.eps = eps

    def initialize(self, x):
        D = x.shape[-1]
        g = _new_param((D,), x.device)
        G.fill_(g.data, 1.0)
        self._param("scale", g, wd_mult=0.0)
        self._param("bias", _new_param((D,), x.device), wd_mult=0.0)

    def forward(self, x):
        return autograd.LayerNorm(self.eps)(x, self.scale, self.bias)


class Pooling2d(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, is_max=True, pad_mode="NOTSET", ceil_mode=False,
                 count_include_pad=True):
        super().__init__()
        self.kernel_size = _pair(kernel_size)
        self.stride = _pair(stride) if stride is not None else self.kernel_size
        self.padding = _pair(padding)
        self.is_max = is_max
        self.pad_mode = pad_mode
        self.ceil_mode = ceil_mode
        self.count_include_pad = count_include_pad

    def forward(self, x):
        return autograd.Pooling2d(self.kernel_size, self.stride, self.padding, self.is_max, self.count_include_pad,
                                  self.ceil_mode)(x)


class MaxPool2d(Pooling2d):
    def __init__(self, kernel_size, stride=None, padding=0, pad_mode="NOTSET", ceil_mode=False):
        super().__init__(kernel_size, stride, padding, True, pad_mode, ceil_mode)


class AvgPool2d(Pooling2d):
    def __init__(self, kernel_size, stride=None, padding=0, pad_mode="NOTSET", ceil_mode=False,
                 count_include_pad=True):
        super().__init__(kernel_size, stride, padding, False, pad_mode, ceil_mode, count_include_pad)


class MaxPool1d(Pooling2d):
    def __init__(self, kernel_size, stride=None, padding=0):
        super().__init__((1, kernel_size), (1, stride or kernel_size), (0, padding), True)


class AvgPool1d(Pooling2d):
    def __init__(self, kernel_size, stride=None, padding=0):
        super().__init__((1, kernel_size), (1, stride or kernel_size), (0, padding), False)


class GlobalAvgPool2d(Layer):
    def __init__(self, keepdims=False):
        super().__init__()
        self.keepdims = keepdims

    def forward(self, x):
        return autograd.GlobalAveragePool(self.keepdims)(x)


class LRN(Layer):
    def __init__(self, size=5, alpha=1e-4, beta=0.75, k=1.0):
        super().__init__()
        self.size, self.alpha, self.beta, self.k = size, alpha, beta, k

    def forward(self, x):
        return autograd.LRN(self.size, self.alpha, self.beta, self.k)(x)


class _Act(Layer):
    op = autograd.Identity

    def forward(self, x):
        return self.op()(x)


class ReLU(_Act):
    op = autograd.ReLU


class Sigmoid(_Act):
    op = autograd.Sigmoid


class Tanh(_Act):
    op = autograd.Tanh


class STanh(_Act):
    op = autograd.STanh


class Gelu(_Act):
    op = autograd.Gelu


class Identity(_Act):
    op = autograd.Identity


class Softmax(Layer):
    def __init__(self, axis=1):
        super().__init__()
        self.axis = axis

    def forward(self, x):
        return autograd.SoftMax(self.axis)(x)


class Add(Layer):
    def forward(self, a, b):
        return autograd.add(a, b)


class Flatten(Layer):
    def __init__(self, axis=1):
        super().__init__()
        self.axis = axis

    def forward(self, x):
        return autograd.Flatten(self.axis)(x)


class Reshape(Layer):
    def forward(self, x, shape):
        return autograd.reshape(x, shape)


class Cat(Layer):
    def __init__(self, axis=0):
        super().__init__()
        self.axis = axis

    def forward(self, xs):
        return autograd.cat(xs, self.axis)


class Dropout(Layer):
    def __init__(self, ratio=0.5):
        super().__init__()
        self.ratio = ratio

    def forward(self, x):
        return autograd.Dropout(self.ratio, x.device)(x)


class SoftMaxCrossEntropy(Layer):
    def __init__(self, topk: int = 1):
        super().__init__()
        self.topk = topk
        self.last_op = None

    def forward(self, x, t):
        op = autograd.SoftMaxCrossEntropy(topk=self.topk)
        self.last_op = op
        return op(x, t)

    def accuracy(self) -> Optional[torch.Tensor]:
        """fp32 device tensor: fraction of the last batch within top-k."""
        return G.reduce(self.last_op.correct, None, "mean", out_dtype=torch.float32) if self.last_op is not None \
            else None


class MeanSquareError(Layer):
    def forward(self, x, t):
        return autograd.MeanSquareError()(x, t)


class CrossEntropy(Layer):
    def forward(self, x, t):
        return autograd.CrossEntropy()(x, t)


class BinaryCrossEntropy(Layer):
    def forward(self, x, t):
        return autograd.BinaryCrossEntropy()(x, t)


class Embedding(Layer):
    def __init__(self, input_dim, output_dim, initializer="gaussian"):
        super().__init__()
        self.input_dim, self.output_dim = input_dim, output_dim

    def initialize(self, x):
        W = _new_param((self.input_dim, self.output_dim), x.device)
        W.gaussian(0.0, 0.02)
        self._param("W", W)

    def forward(self, x):
        return autograd.embedding(x, self.W)


class RNN(Layer):
    """Elman RNN (tanh/relu) unrolled over time with autograd ops."""

    def __init__(self, input_size, hidden_size, num_layers=1, nonlinearity="tanh", bias=True,
                 batch_first=False, dropout=0, bidirectional=False):
        super().__init__()
        self.input_size, self.hidden_size, self.nonlinearity, self.bias = input_size, hidden_size, nonlinearity, bias
        self.batch_first = batch_first

    def initialize(self, xs, h0=None):
        dev = xs.device if isinstance(xs, Tensor) else xs[0].device
        std = math.sqrt(1.0 / self.hidden_size)
        Wx = _new_param((self.input_size, self.hidden_size), dev)
        Wx.uniform(-std, std)
        Wh = _new_param((self.hidden_size, self.hidden_size), dev)
        Wh.uniform(-std, std)
        self._param("Wx", Wx)
        self._param("Wh", Wh)
        self._param("b", _new_param((self.hidden_size,), dev), wd_mult=0.0)

    def forward(self, xs, h0=None):
        if isinstance(xs, Tensor):
            seq = xs.shape[1] if self.batch_first else xs.shape[0]
            steps = [autograd.squeeze(autograd.slice(xs, [t], [t + 1], [1 if self.batch_first else 0]),
                                      1 if self.batch_first else 0) for t in range(seq)]
        else:
            steps = list(xs)
        B = steps[0].shape[0]
        h = h0 if h0 is not None else Tensor((B, self.hidden_size), steps[0].device, requires_grad=False)
        act = autograd.tanh if self.nonlinearity == "tanh" else autograd.relu
        outs = []
        for x in steps:
            h = act(autograd.add(autograd.add(autograd.matmul(x, self.Wx), autograd.matmul(h, self.Wh)), self.b))
            outs.append(h)
        return outs, h


class LSTM(Layer):
    """LSTM unrolled with autograd ops (gates i, f, g, o)."""

    def __init__(self, input_size, hidden_size, nonlinearity="tanh", num_layers=1, bias=True, batch_first=False,
                 dropout=0, bidirectional=False):
        super().__init__()
        self.input_size, self.hidden_size = input_size, hidden_size
        self.batch_first = batch_first

    def initialize(self, xs, hc=None):
        dev = xs.device if isinstance(xs, Tensor) else xs[0].device
        std = math.sqrt(1.0 / self.hidden_size)
        for n, shp in (("Wx", (self.input_size, 4 * self.hidden_size)), ("Wh", (self.hidden_size,
                                                                                4 * self.hidden_size))):
            p = _new_param(shp, dev)
            p.uniform(-std, std)
            self._param(n, p)
        b = _new_param((4 * self.hidden_size,), dev)
        self._param("b", b, wd_mult=0.0)

    def forward(self, xs, hc=None):
        if isinstance(xs, Tensor):
            seq = xs.shape[1] if self.batch_first else xs.shape[0]
            steps = [autograd.squeeze(autograd.slice(xs, [t], [t + 1], [1 if self.batch_first else 0]),
                                      1 if self.batch_first else 0) for t in range(seq)]
        else:
            steps = list(xs)
        B, Hd = steps[0].shape[0], self.hidden_size
        if hc is None:
            h = Tensor((B, Hd), steps[0].device, requires_grad=False)
            c = Tensor((B, Hd), steps[0].device, requires_grad=False)
        else:
            h, c = hc
        outs = []
        for x in steps:
            z = autograd.add(autograd.add(autograd.matmul(x, self.Wx), autograd.matmul(h, self.Wh)), self.b)
            i, f, g, o = autograd.split(z, 1, [Hd, Hd, Hd, Hd])
            i, f, o = autograd.sigmoid(i), autograd.sigmoid(f), autograd.sigmoid(o)
            g = autograd.tanh(g)
            c = autograd.add(autograd.mul(f, c), autograd.mul(i, g))
            h = autograd.mul(o, autograd.tanh(c))
            outs.append(h)
        return outs, (h, c)


CudnnRNN = LSTM
