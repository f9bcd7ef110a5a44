"""Param (reference C11): a trainable tensor created from a ``ParamProto``.

Init methods follow src/utils/param.cc:89-127 exactly (including the
``value`` multiplier and the SqrtFanIn/SqrtFanInOut scalings) and add the
declared-but-unhandled ``kPretrained`` (copy from a checkpoint zip written by
:meth:`singa_amd.model.Model.save_states` or a .npz, looked up by param name).
Learning-rate / weight-decay multipliers travel in ``param_meta`` to the
fused optimiser's per-segment table.  ``fan_in`` for InnerProduct weights is
the input dim (the reference passed in*out: SURVEY Appendix A #7).
"""
from __future__ import annotations

import math
import os
from typing import Optional, Sequence

import numpy as np
import torch

from ..tensor import Tensor

_PRETRAINED_CACHE: dict = {}


def _load_pretrained(path: str) -> dict:
    if path in _PRETRAINED_CACHE:
        return _PRETRAINED_CACHE[path]
    out = {}
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            out = {k: torch.from_numpy(z[k]) for k in z.files}
    else:
        import json
        import zipfile

        from safetensors.torch import load as st_load

        with zipfile.ZipFile(path) as z:
            out = dict(st_load(z.read("tensors.safetensors")))
    _PRETRAINED_CACHE[path] = out
    return out


def init_param(t: Tensor, proto, fan_in: int = 0, generator: Optional[torch.Generator] = None,
               pretrained_path: Optional[str] = None) -> None:
    """Fill ``t`` in place according to a ParamProto."""
    from ..config import schema

    method = schema.enum_name(proto, "init_method")
    shape = t.shape
    d = torch.empty(shape, dtype=torch.float32)
    g = generator
    value = proto.value
    if method == "kConstant":
        d.fill_(value)
    elif method == "kUniform":
        d.uniform_(proto.low, proto.high, generator=g)
        if value:
            d *= value
    elif method == "kUniformSqrtFanIn":
        if fan_in <= 0:
            raise ValueError(f"param {proto.name}: kUniformSqrtFanIn needs fan_in > 0")
        d.uniform_(proto.low, proto.high, generator=g)
        if value:
            d *= value / math.sqrt(fan_in / 3.0)
    elif method == "kUniformSqrtFanInOut":
        d.uniform_(proto.low, proto.high, generator=g)
        if value:
            d *= value / math.sqrt(shape[0] + (shape[1] if len(shape) > 1 else 0))
    elif method == "kGaussain":
        d.normal_(proto.mean, proto.std, generator=g)
        if value:
            d *= value
    elif method == "kGaussainSqrtFanIn":
        d.normal_(proto.mean, proto.std, generator=g)
        if value:
            d *= value / math.sqrt(shape[0])
    elif method == "kPretrained":
        path = pretrained_path or os.environ.get("SINGA_AMD_PRETRAINED")
        if not path:
            raise ValueError(f"param {proto.name}: kPretrained needs a pretrained file")
        src = _load_pretrained(path)
        if proto.name not in src:
            raise KeyError(f"pretrained file has no tensor named {proto.name}")
        d.copy_(src[proto.name].reshape(shape).float())
    else:
        raise ValueError(f"unknown init method {method}")
    from ..ops import glue as G
    G.copy_(t.data, d.reshape(t.data.shape))  # host init + one DMA upload (the native layout pass if strided)


def make_param(shape: Sequence[int], proto, dev, fan_in: int = 0, name: Optional[str] = None,
               generator=None) -> Tensor:
    t = Tensor(tuple(shape), dev, torch.float32, requires_grad=True, stores_grad=True)
    t.name = name or (proto.name if proto is not None and proto.name else None)
    if proto is not None:
        init_param(t, proto, fan_in, generator)
        t.param_meta = {"lr_mult": proto.learning_rate_multiplier, "wd_mult": proto.weight_decay_multiplier}
    else:
        t.param_meta = {"lr_mult": 1.0, "wd_mult": 1.0}
    return t
