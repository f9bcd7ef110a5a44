"""Reference layer catalogue (C21/C22, registered type strings of
src/worker/neuralnet.cc:13-33), executed through singa_amd autograd ops
(and therefore the gfx950 kernels on a RocmGPU).

Every class is registered in :data:`REGISTRY` under the reference type string
("kConvolution", "kInnerProduct", ...).  Layers take their hyper-parameters
from the LayerProto unchanged.  Deliberate fixes of reference quirks
(SURVEY Appendix A): pooling output size uses one formula (floor) for setup
and compute and supports padding (#8); dropout is the identity at test time
(#9); labels are not capped at 10 classes (#10); InnerProduct fan_in is the
input dim (#7); RGBImage reads pixels as unsigned and writes the crop (#12);
Slice/Concate/Split compute for real (#2).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import memory as _mem
from .. import autograd
from ..config import schema
from ..ops import functional as F
from ..ops import glue as G
from ..tensor import Tensor
from .param import make_param

REGISTRY: Dict[str, type] = {}


def register(type_name: str):
    def deco(cls):
        REGISTRY[type_name] = cls
        cls.type_name = type_name
        return cls
    return deco


def create_layer(proto, **kw) -> "RefLayer":
    """Factory<Layer>::Create(type) (reference C18)."""
    try:
        cls = REGISTRY[proto.type]
    except KeyError:
        raise KeyError(f"unknown layer type {proto.type!r} (registered: {sorted(REGISTRY)})")
    return cls(proto, **kw)


class RefLayer:
    type_name = "kBase"
    is_data = False
    is_parser = False
    is_loss = False
    connection = "kOneToOne"  # kOneToAll for layers that read the whole source

    def __init__(self, proto, partition_type: Optional[str] = None):
        self.proto = proto
        self.name = proto.name
        self.srcs: List[str] = list(proto.srclayers)
        pt = partition_type or (schema.enum_name(proto, "partition_type") if proto.HasField("partition_type")
                                else "kNone")
        if self.is_data or self.is_parser:
            pt = "kNone"  # data / parser layers are never partitioned (base_layer.h:359-361)
        self.partition_type = pt
        self.locationid = proto.locationid
        self.partitionid = proto.partitionid
        self.params: List[Tensor] = []
        self.shape: Optional[tuple] = None
        self.dev = None
        self.loss_scale = 1.0   # 1/g for data-partition replicas of a loss

    def partition_dimension(self) -> int:
        return {"kDataPartition": 0, "kLayerPartition": 1}.get(self.partition_type, -1)

    def connection_type(self, i: int) -> str:
        return self.connection

    def setup(self, src_shapes: List[tuple], dev, gen=None) -> tuple:
        self.dev = dev
        self.shape = tuple(src_shapes[0]) if src_shapes else None
        return self.shape

    def forward(self, xs: List, training: bool):
        raise NotImplementedError

    def _pp(self, i: int):
        """i-th ParamProto (defaults if the conf omits it)."""
        if i < len(self.proto.param):
            return self.proto.param[i]
        p = schema.new("ParamProto")
        p.name = f"{self.name}_{'weight' if i == 0 else 'bias'}"
        if i == 0:
            p.init_method = p.kUniformSqrtFanIn
            p.low, p.high, p.value = -1.0, 1.0, 1.0
        return p


# --------------------------------------------------------------------- data
class DataSource:
    """Batches of (images float32 [B, ...], labels int32 [B]) from a Shard
    folder (native Prefetcher thread), an LMDB of Caffe Datums (native
    reader) or a synthetic generator when the path does not exist."""

    def __init__(self, path: str, batch: int, random_skip: int = 0, synthetic_shape=(28, 28), nclass: int = 10,
                 seed: int = 0, loop: bool = True, prefetch: bool = True):
        self.batch = batch
        self.kind = "synthetic"
        self.rng = np.random.RandomState(seed)
        self.shape = tuple(synthetic_shape)
        self.nclass = nclass
        self.prefetcher = None
        if path and os.path.exists(os.path.join(path, "shard.dat")):
            from .. import _core

            sh = _core.Shard(path, _core.kRead)
            first = sh.next()
            if first is None:
                raise ValueError(f"empty shard {path}")
            rec = _core.decode_record(first[1])
            self.shape = tuple(rec["shape"]) if rec["shape"] else (len(rec["data"]) or len(rec["pixel"]),)
            self.dim = int(np.prod(self.shape))
            self.kind = "shard"
            self.prefetcher = _core.Prefetcher(path, batch, self.dim, 1.0, 0.0, loop)
            if random_skip:
                skip = self.rng.randint(0, random_skip + 1) // max(batch, 1)
                buf_i = np.empty((batch, self.dim), np.float32)
                buf_l = np.empty((batch,), np.int32)
                for _ in range(skip):
                    self.prefetcher.next(buf_i, buf_l)
        elif path and os.path.isdir(path) and os.path.exists(os.path.join(path, "data.mdb")):
            self._lmdb_open(path, random_skip)
        self.dim = int(np.prod(self.shape))

    def _lmdb_open(self, path, random_skip=0):
        """Native read-only LMDB cursor (csrc/runtime/lmdb_reader.cc): no
        liblmdb / lmdb module needed.  Values are Caffe Datums
        (reference LMDBDataLayer, src/worker/layer.cc:237-295)."""
        from .. import _core

        self.kind = "lmdb"
        self.cur = _core.LmdbReader(path)
        if self.cur.count() == 0:
            raise ValueError(f"empty LMDB {path}")
        d = _core.decode_datum(self.cur.next()[1])
        if d is None or d["encoded"]:
            raise ValueError(f"{path}: undecodable or encoded (compressed) Datum records are not supported")
        c, h, w = d["shape"]
        self.shape = (c, h, w) if c > 1 else (h, w)
        self.cur.seek_to_first()
        for _ in range(self.rng.randint(0, random_skip + 1) if random_skip else 0):
            if self.cur.next() is None:
                self.cur.seek_to_first()

    def _lmdb_record(self):
        from .. import _core

        kv = self.cur.next()
        if kv is None:  # wrap around (layer.cc:268-274)
            self.cur.seek_to_first()
            kv = self.cur.next()
        d = _core.decode_datum(kv[1])
        px = (np.frombuffer(d["pixel"], np.uint8).astype(np.float32) if d["pixel"]
              else np.asarray(d["data"], np.float32))
        return px.reshape(self.shape), d["label"]

    def next(self):
        B = self.batch
        if self.kind == "shard":
            img = np.empty((B, self.dim), np.float32)
            lab = np.empty((B,), np.int32)
            n = self.prefetcher.next(img, lab)
            return img[:n].reshape((n,) + self.shape), lab[:n]
        if self.kind == "lmdb":
            recs = [self._lmdb_record() for _ in range(B)]
            return np.stack([r[0] for r in recs]), np.asarray([r[1] for r in recs], np.int32)
        img = self.rng.randint(0, 256, size=(B,) + self.shape).astype(np.float32)
        lab = self.rng.randint(0, self.nclass, size=(B,)).astype(np.int32)
        return img, lab


class _DataLayerBase(RefLayer):
    is_data = True

    def configure(self, synthetic_shape=(28, 28), nclass=10, seed=0, prefetch=True):
        dp = self.proto.data_param
        self.batch = int(dp.batchsize) if dp.batchsize else 64
        self.source = DataSource(dp.path, self.batch, dp.random_skip, synthetic_shape, nclass, seed,
                                 prefetch=prefetch)
        self.sample_shape = self.source.shape

    def setup(self, src_shapes, dev, gen=None):
        self.dev = dev
        if not hasattr(self, "source"):
            self.configure()
        self.shape = (self.batch,) + tuple(self.sample_shape)
        return self.shape

    def forward(self, xs, training):
        img, lab = self.source.next()
        self.draws = getattr(self, "draws", 0) + 1  # batches consumed (checkpoint fast-forward)
        return {"image": Tensor(device=self.dev, data=torch.from_numpy(np.ascontiguousarray(img)),
                                requires_grad=False),
                "label": Tensor(device=self.dev, data=torch.from_numpy(lab), requires_grad=False)}


@register("kShardData")
class ShardDataLayer(_DataLayerBase):
    pass


@register("kLMDBData")
class LMDBDataLayer(_DataLayerBase):
    pass


@register("kSyntheticData")
class SyntheticDataLayer(_DataLayerBase):
    pass


@register("kMnistImage")
class MnistImageLayer(RefLayer):
    """MNIST parser: ``x / norm_a - norm_b`` (optionally resized), plus the
    training-time deformations that ``MnistProto`` describes.  The reference
    parses the fields but leaves the transform commented out
    (``src/worker/layer.cc:405-436``); this implements the intent, batched on
    the layer's device with one ``grid_sample``:

    * ``gamma`` — per-axis scaling by ``1 + r*gamma/100``, ``r ~ U(-1, 1)``;
    * ``beta``  — per image, either a rotation by ``r*beta`` degrees or a
      horizontal shear ``r*beta/90`` (halved for the digits 1 and 7);
    * ``kernel``/``sigma``/``alpha`` — elastic distortion (Simard et al.):
      uniform random displacement fields smoothed by a ``kernel``-wide
      Gaussian of std ``sigma`` and scaled to ``alpha`` pixels, applied to
      every ``elastic_freq``-th batch (every batch when 0).

    All fields default to 0, i.e. no augmentation, as in the reference.
    """
    is_parser = True

    def setup(self, src_shapes, dev, gen=None):
        self.dev = dev
        mp = self.proto.mnist_param
        self.norm_a, self.norm_b = mp.norm_a or 1.0, mp.norm_b
        self.resize = mp.resize
        self.gamma, self.beta = float(mp.gamma), float(mp.beta)
        self.kernel, self.sigma, self.alpha = int(mp.kernel), float(mp.sigma), float(mp.alpha)
        self.elastic_freq = int(mp.elastic_freq)
        self.nbatch = 0
        self.rng = np.random.RandomState(0)
        B = src_shapes[0][0]
        s = src_shapes[0][1:]
        self.shape = (B, self.resize, self.resize) if self.resize else (B,) + tuple(s)
        return self.shape

    def _rand(self, *shape) -> np.ndarray:
        return self.rng.uniform(-1.0, 1.0, size=shape).astype(np.float32)

    def _theta(self, B: int, label) -> np.ndarray:
        """Per-image affine sampling matrices [B][2][3] (host scalars)."""
        theta = np.zeros((B, 2, 3), np.float32)
        theta[:, 0, 0] = theta[:, 1, 1] = 1.0
        if self.gamma > 0:  # scaling the image by s = sampling coordinates by 1/s
            theta[:, 0, 0] = 1.0 / (1.0 + self._rand(B) * self.gamma / 100.0)
            theta[:, 1, 1] = 1.0 / (1.0 + self._rand(B) * self.gamma / 100.0)
        if self.beta > 0:
            r = self._rand(B)
            rot = self.rng.uniform(0.0, 1.0, size=B) < 0.5
            ang = np.deg2rad(r * self.beta)
            c, sn = np.cos(ang), np.sin(ang)
            R = np.zeros((B, 2, 2), np.float32)
            R[:, 0, 0], R[:, 0, 1], R[:, 1, 0], R[:, 1, 1] = c, -sn, sn, c
            sh = r * self.beta / 90.0
            if label is not None:
                lab = np.asarray(label).reshape(-1)
                sh = np.where((lab == 1) | (lab == 7), sh / 2, sh)
            S = np.tile(np.eye(2, dtype=np.float32), (B, 1, 1))
            S[:, 0, 1] = sh
            A = np.where(rot[:, None, None], R, S)
            theta[:, :, :2] = A @ theta[:, :, :2]
        return np.ascontiguousarray(theta, np.float32)

    def _deform(self, img: np.ndarray, label) -> np.ndarray:
        """img [B, H, W] float32 (host) -> deformed [B, H, W]: bilinear
        sampling through the affine map plus (elastic) a Gaussian-smoothed
        random displacement field, zero outside -- all on the native C++
        host kernels (csrc/runtime/cpu_ops.cc AffineElasticSample /
        GaussBlur2D)."""
        B, H, W = img.shape
        use_affine = self.gamma > 0 or self.beta > 0
        use_elastic = self.alpha > 0 and self.kernel > 0 and self.sigma > 0 and \
            (self.elastic_freq <= 0 or self.nbatch % self.elastic_freq == 0)
        if not (use_affine or use_elastic):
            return img
        from ..ops import cpu as CP
        C = CP.lib()
        theta = self._theta(B, label)
        disp = None
        if use_elastic:
            k = self.kernel | 1
            ax = np.arange(k, dtype=np.float32) - k // 2
            g1 = np.exp(-ax ** 2 / (2 * self.sigma ** 2)).astype(np.float32)
            g1 /= g1.sum()
            d = self._rand(B * 2, H, W)
            sm = np.empty_like(d)
            C.gauss_blur2d(d.ctypes.data, sm.ctypes.data, B * 2, H, W, g1.ctypes.data, k)
            # alpha pixels -> normalised [-1, 1] grid units, interleaved (dx, dy)
            disp = np.ascontiguousarray(np.stack([sm.reshape(B, 2, H, W)[:, 0] * (self.alpha * 2.0 / W),
                                                  sm.reshape(B, 2, H, W)[:, 1] * (self.alpha * 2.0 / H)], -1),
                                        np.float32)
        out = np.empty_like(img)
        C.affine_elastic_sample(img.ctypes.data, theta.ctypes.data, 0 if disp is None else disp.ctypes.data,
                                out.ctypes.data, B, H, W)
        return out

    def forward(self, xs, training):
        src = xs[0]["image"].data
        dev = self.dev.torch_device  # (singa device: no tensor-attribute query on the hot path)
        aug = training and (self.gamma > 0 or self.beta > 0 or (self.alpha > 0 and self.kernel > 0 and self.sigma > 0))
        need_resize = bool(self.resize) and tuple(src.shape[-2:]) != (self.resize, self.resize)
        if aug or need_resize:
            # resize / affine / elastic augmentation is host-side preprocessing
            # (the reference's CPU parser, src/worker/layer.cc:382-473) on the
            # native C++ kernels; a GPU batch comes back with one upload
            from ..ops import cpu as CP
            img = np.ascontiguousarray(G.to(src, torch.float32).cpu().numpy(), np.float32)
            if img.ndim == 2:
                img = img[None]
            img = img.reshape(img.shape[0], img.shape[-2], img.shape[-1])
            if need_resize:
                r = np.empty((img.shape[0], self.resize, self.resize), np.float32)
                CP.lib().resize_bilinear(img.ctypes.data, r.ctypes.data, img.shape[0], img.shape[1], img.shape[2],
                                         self.resize, self.resize)
                img = r
            if training:
                lab = xs[0].get("label") if isinstance(xs[0], dict) else None
                img = self._deform(img, lab.data.cpu().numpy() if lab is not None else None)
                self.nbatch += 1
            t = torch.from_numpy(img)
            imgt = t if dev.type == "cpu" else G.copy_(_mem.empty(tuple(t.shape), dtype=torch.float32, device=dev), t)
        else:
            imgt = G.to(src, torch.float32)
            if training:
                self.nbatch += 1
        # x / norm_a - norm_b
        out = F.unary("adds", F.unary("scale", imgt, 1.0 / self.norm_a), -float(self.norm_b))
        return Tensor(device=self.dev, data=out, requires_grad=False)


@register("kRGBImage")
class RGBImageLayer(RefLayer):
    is_parser = True

    def setup(self, src_shapes, dev, gen=None):
        self.dev = dev
        rp = self.proto.rgbimage_param
        self.scale, self.crop, self.mirror = rp.scale, rp.cropsize, rp.mirror
        B, C, H, W = src_shapes[0]
        self.shape = (B, C, self.crop, self.crop) if self.crop else (B, C, H, W)
        self.rng = np.random.RandomState(0)
        return self.shape

    def forward(self, xs, training):
        img = G.to(xs[0]["image"].data, torch.float32)
        if self.crop:
            H, W = img.shape[-2:]
            if training:
                h0, w0 = self.rng.randint(0, H - self.crop + 1), self.rng.randint(0, W - self.crop + 1)
            else:
                h0, w0 = (H - self.crop) // 2, (W - self.crop) // 2
            img = img[..., h0:h0 + self.crop, w0:w0 + self.crop]
        if self.mirror and training and self.rng.randint(2):  # horizontal mirror: a reversed-index gather
            W = img.shape[-1]
            key = (W, str(img.device))
            rev = self._rev.get(key) if hasattr(self, "_rev") else None
            if rev is None:
                self._rev = getattr(self, "_rev", {})
                rev = self._rev[key] = torch.arange(W - 1, -1, -1, dtype=torch.int64).to(img.device)
            img = G.index_select(img, img.dim() - 1, rev)
        return Tensor(device=self.dev, data=F.unary("scale", G.contiguous(img), float(self.scale)),
                      requires_grad=False)


@register("kLabel")
class LabelLayer(RefLayer):
    is_parser = True

    def setup(self, src_shapes, dev, gen=None):
        self.dev = dev
        self.shape = (src_shapes[0][0],)
        return self.shape

    def forward(self, xs, training):
        return xs[0]["label"]


# ------------------------------------------------------------------- neurons
@register("kConvolution")
class ConvolutionLayer(RefLayer):
    connection = "kOneToAll"

    def setup(self, src_shapes, dev, gen=None):
        self.dev = dev
        cp = self.proto.convolution_param
        s = src_shapes[0]
        C = s[-3] if len(s) > 3 else 1
        H, W = s[-2], s[-1]
        self.k, self.pad, self.stride = cp.kernel, cp.pad, cp.stride
        self.nf = getattr(self, "nf_override", None) or cp.num_filters
        self.bias = cp.bias_term
        Ho = (H + 2 * self.pad - self.k) // self.stride + 1
        Wo = (W + 2 * self.pad - self.k) // self.stride + 1
        self.in_c = C
        if not self.params:
            w = make_param((self.nf, C, self.k, self.k), self._pp(0), dev, fan_in=C * self.k * self.k,
                           name=f"{self.name}/weight", generator=gen)
            self.params = [w]
            if self.bias:
                self.params.append(make_param((self.nf,), self._pp(1), dev, name=f"{self.name}/bias",
                                              generator=gen))
        self.shape = (s[0], self.nf, Ho, Wo)
        return self.shape

    def forward(self, xs, training):
        x = xs[0]
        if x.ndim() == 3:
            x = autograd.reshape(x, (x.shape[0], 1, x.shape[1], x.shape[2]))
        op = autograd.Conv2d((self.stride, self.stride), (self.pad, self.pad), has_bias=self.bias)
        return op(x, *self.params)


@register("kInnerProduct")
class InnerProductLayer(RefLayer):
    connection = "kOneToAll"

    def setup(self, src_shapes, dev, gen=None):
        self.dev = dev
        s = src_shapes[0]
        self.vdim = int(np.prod(s[1:]))
        self.hdim = getattr(self, "nf_override", None) or self.proto.inner_product_param.num_output
        self.bias = self.proto.inner_product_param.bias_term
        if not self.params:
            self.params = [make_param((self.vdim, self.hdim), self._pp(0), dev, fan_in=self.vdim,
                                      name=f"{self.name}/weight", generator=gen)]
            if self.bias:
                self.params.append(make_param((self.hdim,), self._pp(1), dev, name=f"{self.name}/bias",
                                              generator=gen))
        self.shape = (s[0], self.hdim)
        return self.shape

    def forward(self, xs, training):
        x = xs[0]
        if x.ndim() != 2:
            x = autograd.reshape(x, (x.shape[0], -1))
        return autograd.Linear(self.bias)(x, *self.params)


@register("kPooling")
class PoolingLayer(RefLayer):
    def setup(self, src_shapes, dev, gen=None):
        self.dev = dev
        pp = self.proto.pooling_param
        self.k, self.stride, self.pad = pp.kernel, pp.stride, pp.pad
        self.is_max = schema.enum_name(pp, "pool") == "MAX"
        s = src_shapes[0]
        Ho = (s[-2] + 2 * self.pad - self.k) // self.stride + 1
        Wo = (s[-1] + 2 * self.pad - self.k) // self.stride + 1
        self.shape = tuple(s[:-2]) + (Ho, Wo)
        return self.shape

    def forward(self, xs, training):
        return autograd.Pooling2d((self.k, self.k), (self.stride, self.stride), (self.pad, self.pad),
                                  self.is_max, count_include_pad=True)(xs[0])


@register("kReLU")
class ReLULayer(RefLayer):
    def forward(self, xs, training):
        ns = self.proto.relu_param.negative_slope
        return autograd.leakyrelu(xs[0], ns) if ns else autograd.relu(xs[0])


@register("kTanh")
class TanhLayer(RefLayer):
    def forward(self, xs, training):
        tp = self.proto.tanh_param
        if self.proto.HasField("tanh_param") and (tp.HasField("outer_scale") or tp.HasField("inner_scale")):
            y = autograd.tanh(autograd.mul(xs[0], float(tp.inner_scale)))
            return autograd.mul(y, float(tp.outer_scale))
        return autograd.stanh(xs[0])


@register("kDropout")
class DropoutLayer(RefLayer):
    def forward(self, xs, training):
        if not training:
            return xs[0]
        return autograd.Dropout(self.proto.dropout_param.dropout_ratio, xs[0].device)(xs[0])


@register("kLRN")
class LRNLayer(RefLayer):
    def forward(self, xs, training):
        lp = self.proto.lrn_param
        return autograd.LRN(lp.local_size, lp.alpha, lp.beta, lp.knorm)(xs[0])


@register("kSoftmaxLoss")
class SoftmaxLossLayer(RefLayer):
    is_loss = True
    connection = "kOneToAll"

    def __init__(self, proto, partition_type=None):
        super().__init__(proto, partition_type)
        if self.partition_type == "kLayerPartition":
            self.partition_type = "kNone"  # include/worker/layer.h:216-221

    def setup(self, src_shapes, dev, gen=None):
        self.dev = dev
        self.topk = self.proto.softmaxloss_param.topk
        self.scale = self.proto.softmaxloss_param.scale
        self.shape = (2,)
        return self.shape

    def forward(self, xs, training):
        x, lab = xs[0], xs[1]
        if x.ndim() != 2:
            x = autograd.reshape(x, (x.shape[0], -1))
        op = autograd.SoftMaxCrossEntropy(topk=self.topk)
        loss = op(x, lab)
        self.metric = (F.unary("scale", loss.data.detach(), float(self.scale)),
                       F.unary("scale", G.reduce(op.correct, None, "mean", out_dtype=torch.float32), float(self.scale)))
        s = self.scale * self.loss_scale
        if s != 1.0:
            loss = autograd.mul(loss, s)
        return loss


# -------------------------------------------------------------- connection
@register("kSplit")
class SplitLayer(RefLayer):
    def forward(self, xs, training):
        return autograd.identity(xs[0])


@register("kSlice")
class SliceLayer(RefLayer):
    """Splits along slice_dimension into slice_num parts; the last part takes
    the remainder (src/worker/base_layer.cc:125-132).  Output j feeds dst j."""

    def setup(self, src_shapes, dev, gen=None):
        self.dev = dev
        sp = self.proto.slice_param
        self.dim, self.num = sp.slice_dimension, max(1, sp.slice_num)
        s = list(src_shapes[0])
        n = s[self.dim]
        base = n // self.num
        self.sizes = [base] * (self.num - 1) + [n - base * (self.num - 1)]
        self.shapes = []
        for k in self.sizes:
            t = list(s)
            t[self.dim] = k
            self.shapes.append(tuple(t))
        self.shape = tuple(s)
        return self.shape

    def forward(self, xs, training):
        x = xs[0]
        n = x.shape[self.dim]
        if sum(self.sizes) != n:  # a micro-batch (pipelined step): same rule on the actual size
            base = n // self.num
            self.sizes = [base] * (self.num - 1) + [n - base * (self.num - 1)]
        if x.requires_grad:
            parts = autograd.split(x, self.dim, self.sizes)
        else:
            parts = tuple(Tensor(device=x.device, data=p, requires_grad=False)
                          for p in torch.split(x.data, self.sizes, dim=self.dim))
        return list(parts) if isinstance(parts, tuple) else [parts]


@register("kConcate")
class ConcateLayer(RefLayer):
    def setup(self, src_shapes, dev, gen=None):
        self.dev = dev
        self.dim = self.proto.concate_param.concate_dimension
        s = list(src_shapes[0])
        s[self.dim] = sum(t[self.dim] for t in src_shapes)
        self.shape = tuple(s)
        return self.shape

    def forward(self, xs, training):
        if any(x.requires_grad for x in xs):
            return autograd.cat(xs, self.dim)
        return Tensor(device=xs[0].device, data=G.cat([x.data for x in xs], self.dim), requires_grad=False)


@register("kBridgeSrc")
class BridgeSrcLayer(RefLayer):
    """Ships activations to another location (device); gradients come back
    through autograd.  In one process locations map to devices; across
    processes see singa_amd.parallel.pipeline."""

    def forward(self, xs, training):
        return autograd.identity(xs[0]) if xs[0].requires_grad else xs[0]


@register("kBridgeDst")
class BridgeDstLayer(BridgeSrcLayer):
    pass
