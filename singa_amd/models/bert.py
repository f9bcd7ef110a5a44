"""BERT encoder (Devlin et al. 2019) -- the north-star ``sonnx`` model
family (SURVEY §7.2 phase 10: MatMul, Softmax, LayerNorm, GELU, Add,
Reshape/Transpose, Gather).  BERT-base: 12 layers, hidden 768, 12 heads,
FFN 3072, vocab 30522, 512 positions.

GPU bf16 path: every projection is the MFMA GEMM with a fused bias epilogue,
attention is batched MFMA GEMMs + the softmax kernels (autograd.Attention),
LayerNorm / GELU / dropout are the hand-written kernels; fp32 master weights
in the flat ParamStore.
"""
from __future__ import annotations

import os

import math
from typing import Optional

import torch

from .. import autograd, layer, model
from ..tensor import Tensor
from ..ops import functional as F
from ..ops import glue as G


_IDS: dict = {}


def _const_ids(S: int, device, kind: str) -> torch.Tensor:
    """[1, S] position ids (0..S-1) or zero type ids, built once per (S,
    device) on the host and uploaded (a plain DMA copy): the step launches
    no kernel for them."""
    key = (S, str(device), kind)
    t = _IDS.get(key)
    if t is None:
        import numpy as np
        h = np.arange(S, dtype=np.int64)[None] if kind == "pos" else np.zeros((1, S), np.int64)
        t = _IDS[key] = torch.from_numpy(h).to(device)
    return t


class SplitHeads(autograd.Operator):
    """[B, S, 3*H*D] -> q, k, v each [B, H, S, D] (contiguous)."""

    def __init__(self, heads: int, name=None):
        super().__init__(name)
        self.h = heads

    def forward(self, x):
        B, S, E3 = x.shape
        D = E3 // (3 * self.h)
        # one permuting copy; q, k, v are contiguous slices of it
        t = G.contiguous(x.view(B, S, 3, self.h, D).permute(2, 0, 3, 1, 4))
        return t[0], t[1], t[2]

    def backward(self, dq, dk, dv):
        ref = next(d for d in (dq, dk, dv) if d is not None)
        B, H, S, D = ref.shape
        parts = [(d if d is not None else G.zeros_like(ref)).unsqueeze(0) for d in (dq, dk, dv)]
        return G.reshape(G.contiguous(G.cat(parts, 0).permute(1, 3, 0, 2, 4)), (B, S, 3 * H * D))


class MergeHeads(autograd.Operator):
    """[B, H, S, D] -> [B, S, H*D]."""

    def forward(self, x):
        B, H, S, D = x.shape
        return G.reshape(G.contiguous(x.permute(0, 2, 1, 3)), (B, S, H * D))

    def backward(self, dy):
        B, S, E = dy.shape
        H = self.h
        return G.contiguous(G.reshape(dy, (B, S, H, E // H)).permute(0, 2, 1, 3))

    def __call__(self, x):
        self.h = x.shape[1]
        return super().__call__(x)


def _drop_add_ln(x, a, drop: layer.Dropout, ln: layer.LayerNorm):
    """ln(x + drop(a)): one fused operator on the GPU (autograd.DropAddLayerNorm,
    same numbers; SINGA_AMD_FUSED_DAL=0 disables), the three layers otherwise
    (and while tracing an ONNX export, which keeps the standard nodes)."""
    if (os.environ.get("SINGA_AMD_FUSED_DAL", "1") != "0" and not autograd._TRACE and x.data.is_cuda
            and F.drop_add_ln_ok(x.data, a.data)):
        if not ln._initialized:
            ln.initialize(x)
            ln._initialized = True
        return autograd.DropAddLayerNorm(drop.ratio, x.device, ln.eps)(x, a, ln.scale, ln.bias)
    return ln(autograd.add(x, drop(a)))


class EncoderLayer(layer.Layer):
    def __init__(self, hidden: int, heads: int, ffn: int, dropout: float = 0.1, fuse_gelu: Optional[bool] = None):
        super().__init__()
        if fuse_gelu is None:
            fuse_gelu = os.environ.get("SINGA_AMD_FUSE_GELU", "0") != "0"
        self.heads = heads
        self.qkv = layer.Linear(3 * hidden)
        self.proj = layer.Linear(hidden)
        self.ln1 = layer.LayerNorm(1e-12)
        # fuse_gelu (SINGA_AMD_FUSE_GELU=1): GELU in fc1's GEMM epilogue (forward)
        # and fc2's data-gradient epilogue (backward).  Off by default: measured
        # neutral-to-slower (3373-3381 vs 3383-3384 seq/s, sonnx 3240-3242 vs
        # 3245-3254, profiles/r4/ab_gelu_fusion.jsonl) -- the erf in the epilogue
        # is exposed work there, hidden behind memory in the separate kernel
        self.fc1 = layer.Linear(ffn, activation="gelu" if fuse_gelu else None)
        self.act = layer.Identity() if fuse_gelu else layer.Gelu()
        self.fc2 = layer.Linear(hidden)
        self.ln2 = layer.LayerNorm(1e-12)
        self.drop1 = layer.Dropout(dropout)
        self.drop2 = layer.Dropout(dropout)

    def forward(self, x, mask: Optional[Tensor] = None):
        qkv = self.qkv(x)
        att = autograd.QKVAttention(self.heads)  # heads addressed in place: no split / merge copies
        a = att(qkv, mask) if mask is not None else att(qkv)
        x = _drop_add_ln(x, self.proj(a), self.drop1, self.ln1)
        return _drop_add_ln(x, self.fc2(self.act(self.fc1(x))), self.drop2, self.ln2)


class Embeddings(layer.Layer):
    def __init__(self, vocab: int, hidden: int, max_pos: int, type_vocab: int, dropout: float):
        super().__init__()
        self.vocab, self.hidden, self.max_pos, self.type_vocab = vocab, hidden, max_pos, type_vocab
        self.ln = layer.LayerNorm(1e-12)
        self.drop = layer.Dropout(dropout)

    def initialize(self, ids, types=None):
        dev = ids.device
        for name, n in (("word", self.vocab), ("position", self.max_pos), ("token_type", self.type_vocab)):
            W = Tensor((n, self.hidden), dev, requires_grad=True, stores_grad=True)
            W.gaussian(0.0, 0.02)
            self._param(name, W, wd_mult=0.0)

    def forward(self, ids, types=None):
        B, S = ids.shape
        # [1, S] position / type ids broadcast over the batch (an exported
        # ONNX graph stays batch-size independent)
        pos = Tensor(data=_const_ids(S, ids.data.device, "pos"), device=ids.device, requires_grad=False)
        e = autograd.add(autograd.embedding(ids, self.word), autograd.embedding(pos, self.position))
        if types is None:
            types = Tensor(data=_const_ids(S, ids.data.device, "zero"), device=ids.device, requires_grad=False)
        e = autograd.add(e, autograd.embedding(types, self.token_type))
        return self.drop(self.ln(e))


class Bert(model.Model):
    def __init__(self, vocab: int = 30522, hidden: int = 768, layers: int = 12, heads: int = 12, ffn: int = 3072,
                 max_pos: int = 512, type_vocab: int = 2, num_labels: int = 2, dropout: float = 0.1,
                 compute_dtype=torch.bfloat16):
        super().__init__()
        self.compute_dtype = compute_dtype
        self.embeddings = Embeddings(vocab, hidden, max_pos, type_vocab, dropout)
        self.encoder = [EncoderLayer(hidden, heads, ffn, dropout) for _ in range(layers)]
        self.pooler = layer.Linear(hidden)
        self.pool_act = layer.Tanh()
        self.classifier = layer.Linear(num_labels)
        self.loss_fn = layer.SoftMaxCrossEntropy()

    def encode(self, ids, mask=None, types=None):
        x = self.embeddings(ids, types)
        if x.data.is_cuda and x.dtype != self.compute_dtype:
            x = autograd.cast(x, self.compute_dtype)
        m = None
        if mask is not None:  # [B, S] of 1/0 -> additive [B, 1, 1, S]
            md = mask.data if isinstance(mask, Tensor) else mask
            add = G.binary("mul", G.binary("sub", G.full((), 1.0, torch.float32, md.device), G.to(md, torch.float32)),
                           -10000.0)
            m = Tensor(data=add.view(md.shape[0], 1, 1, md.shape[1]), device=ids.device, requires_grad=False)
        for blk in self.encoder:
            x = blk(x, m)
        return x

    def forward(self, ids, mask=None, types=None):
        x = self.encode(ids, mask, types)
        cls = TorchCLS()(x)
        return self.classifier(self.pool_act(self.pooler(cls)))

    def train_one_batch(self, ids, y, mask=None):
        out = self.forward(ids, mask)
        loss = self.loss_fn(out, y)
        self.optimizer(loss)
        return out, loss


class TorchCLS(autograd.Operator):
    """x[:, 0] (the [CLS] token)."""

    def forward(self, x):
        self.shape = x.shape
        return G.contiguous(x[:, 0])

    def backward(self, dy):
        dx = G.zeros(self.shape, dy.dtype, dy.device)
        G.copy_(dx[:, 0], dy)
        return dx


def bert_base(**kw) -> Bert:
    return Bert(**kw)


def bert_tiny(**kw) -> Bert:
    kw = {**dict(vocab=1000, hidden=128, layers=2, heads=2, ffn=512, max_pos=128), **kw}
    return Bert(**kw)


def create_model(size: str = "base", **kw) -> Bert:
    return bert_base(**kw) if size == "base" else bert_tiny(**kw)
