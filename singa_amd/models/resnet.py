"""ResNet (v1.5: stride on the 3x3 conv) for ImageNet-shaped input.

The flagship benchmark model (BASELINE.json: "ResNet-50 bf16 training").
Built from :mod:`singa_amd.layer` layers with the MI355X-oriented fusions:

* the input batch (fp32 NCHW) enters through one HIP kernel that writes bf16
  NHWC with channels zero-padded 3 -> 8 (16-byte vectors for the stem conv's
  implicit-GEMM loader); the stem weight keeps its logical 3 input channels;
* every conv -> BN -> ReLU is conv + one fused BN-apply(+ReLU) pass, and the
  block output BN -> (+identity) -> ReLU is one fused pass as well; their
  backward passes reuse the saved block output as the ReLU mask;
* bf16 activations, fp32 master weights in the flat ParamStore, fp32 BN
  statistics and loss.

The reference has no ResNet, BatchNorm or bf16; this model is a
north-star addition.
"""
from __future__ import annotations

import os
from types import SimpleNamespace
from typing import List, Sequence

import torch

from .. import memory as _mem
from .. import autograd, layer, model
from ..ops import functional as F
from ..ops import native as N
from ..tensor import Tensor
from ..ops import glue as G


class InputPrep(autograd.Operator):
    """fp32 NCHW -> compute dtype NHWC (channels padded to a multiple of 8 on GPU)."""

    def __init__(self, dtype=torch.bfloat16, name=None):
        super().__init__(name)
        self.dtype = dtype

    def forward(self, x):
        if x.is_cuda and x.dim() == 4:
            C = x.shape[1]
            cp = (C + 7) // 8 * 8
            if x.dtype == torch.float32 and self.dtype == torch.bfloat16 and x.is_contiguous():
                y = _mem.empty((x.shape[0], cp, x.shape[2], x.shape[3]), dtype=torch.bfloat16, device=x.device,
                                memory_format=torch.channels_last)
                N.lib().nchw_to_nhwc_pad(x.data_ptr(), y.data_ptr(), x.shape[0], C, x.shape[2], x.shape[3], cp,
                                         N.stream())
                return y
            return F.to_nhwc_bf16(x, cp) if self.dtype == torch.bfloat16 else G.to(
                x, memory_format=torch.channels_last)
        return G.to(x, self.dtype) if x.dtype != self.dtype else x

    def backward(self, dy):
        return None


_PAIR_IDX: dict = {}


def _pair_maps(K: int, C: int, device):
    """Index maps between the stem filter W [K][7][7][C] (KRSC flat, C <= 3)
    and its paired-tap form W' [K][7][4][8]: W'[k][r][j][c'] = W[k][r][2j][c']
    (c' < 3), W[k][r][2j+1][c'-3] (3 <= c' < 6, 2j+1 < 7), else 0.
    fwd: W' = cat(W_flat, 0)[fwd]; bwd: dW_flat = dW'_flat[bwd]."""
    key = (K, C, str(device))
    if key not in _PAIR_IDX:
        zero = K * 49 * C
        fwd = torch.full((K, 7, 4, 8), zero, dtype=torch.int64)
        bwd = _mem.empty((K, 7, 7, C), dtype=torch.int64)
        k = torch.arange(K).view(K, 1)
        r = torch.arange(7).view(1, 7)
        for s in range(7):
            j, half = s // 2, s % 2
            for c in range(C):
                src = k * 49 * C + r * 7 * C + s * C + c
                dst = ((k * 7 + r) * 4 + j) * 8 + half * 3 + c
                fwd.view(-1)[dst.reshape(-1)] = src.reshape(-1)
                bwd[:, :, s, c] = dst
        _PAIR_IDX[key] = (fwd.view(-1).to(device), bwd.view(-1).to(device))
    return _PAIR_IDX[key]


class PairedStemConv(autograd.Operator):
    """The 7x7 / stride-2 / pad-3 ImageNet stem over <= 3 input channels
    (fp32 NCHW batch in, bf16 NHWC out), run as a 7x4 conv with horizontal
    dilation 2 over the "paired-tap" input (``nchw_to_pairs``: each 16-byte
    pixel vector holds two horizontally adjacent pixels): 224 reduction
    elements per output instead of 392 with 3 -> 8 channel padding, and half
    the implicit-GEMM gather vectors -- forward and weight gradient.  The
    input needs no gradient (it is the data)."""

    def __init__(self, bn_stats: bool = False, name=None):
        super().__init__(name)
        self.bn_stats = bn_stats

    @staticmethod
    def applies(x, w_shape) -> bool:
        return (x.is_cuda and x.dim() == 4 and x.dtype == torch.float32 and x.is_contiguous()
                and x.shape[1] <= 3 and tuple(w_shape[1:]) == (x.shape[1], 7, 7) and N.available()
                and not autograd._TRACE)

    def forward(self, x, W):
        L = N.lib()
        Nn, C, H, Wd = x.shape
        K = W.shape[0]
        xp = _mem.empty((Nn, H, Wd + 1, 8), dtype=torch.bfloat16, device=x.device)
        L.nchw_to_pairs(x.data_ptr(), xp.data_ptr(), Nn, C, H, Wd, N.stream())
        p = self.params[1] if len(self.params) > 1 else None
        low = p.low if p is not None else None
        wk = G.reshape((low if low is not None else G.to(W, torch.bfloat16)).permute(0, 2, 3, 1), (-1,))  # KRSC
        fwd, bwd = _pair_maps(K, C, x.device)
        wp = G.index_select(G.cat([wk, G.zeros((1,), torch.bfloat16, x.device)]), 0, fwd)
        Ho, Wo = (H + 6 - 7) // 2 + 1, (Wd + 6 - 7) // 2 + 1
        y = _mem.empty((Nn, K, Ho, Wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        ws, rows = None, 0
        if self.bn_stats and autograd.training:
            rows = L.conv_stats_rows(Nn * Ho * Wo, K)
            if rows > 0:
                ws = F.zeroed_ws(rows * 2 * K, x.device)
        # the persistent stem kernel (csrc/kernels/stem.hip: filters and input rows
        # staged once in LDS), else the generic conv in the paired geometry:
        # width Wd+1, S = 4 taps of dilation 2, pad (3, 2)
        if not (K == 64 and (rows == 32 or ws is None) and os.environ.get("SINGA_AMD_STEM_KERNEL", "1") != "0"
                and L.stem_fwd(xp.data_ptr(), wp.data_ptr(), y.data_ptr(), N.ptr(ws), Nn, H, Wd + 1, Ho, Wo,
                               N.stream())):
            L.conv_fwd(xp.data_ptr(), wp.data_ptr(), y.data_ptr(), 0, Nn, H, Wd + 1, 8, K, 7, 4, Ho, Wo, 2, 2, 3, 2, 1,
                       2, 0, 0, N.stream(), N.ptr(ws))
        if ws is not None:
            y._sg_bn_ws = (ws, rows)
        if self.requires_grad:
            self.xp, self.shape = xp, (Nn, C, H, Wd, K, Ho, Wo)
        return y

    def backward(self, dy):
        L = N.lib()
        Nn, C, H, Wd, K, Ho, Wo = self.shape
        xp, self.xp = self.xp, None
        if not (dy.dtype == torch.bfloat16 and N.is_cl(dy)):
            dy = G.to(dy, torch.bfloat16, torch.channels_last)
        dwp = G.zeros((K * 7 * 4 * 8,), torch.float32, dy.device)
        L.conv_wgrad(xp.data_ptr(), dy.data_ptr(), dwp.data_ptr(), Nn, H, Wd + 1, 8, K, 7, 4, Ho, Wo, 2, 2, 3, 2, 1,
                     2, 0, N.stream())
        _, bwd = _pair_maps(K, C, dy.device)
        dw = G.index_select(dwp, 0, bwd).view(K, 7, 7, C).permute(0, 3, 1, 2)  # logical KCRS
        tgt = self.grad_target(1)
        if tgt is not None:
            G.binary("add", tgt, dw, out=tgt)
            return None, autograd.ACCUMULATED
        return None, G.contiguous(dw)


class StemConv2d(layer.Conv2d):
    """ResNet stem conv (7x7/2, pad 3) fed the raw fp32 NCHW batch: the
    paired-tap HIP path for bf16 on GPU (:class:`PairedStemConv`; disable with
    ``SINGA_PAIRED_STEM=0``), otherwise :class:`InputPrep` + the generic conv."""

    compute_dtype = torch.bfloat16

    def forward(self, x):
        dt = self.compute_dtype if x.data.is_cuda else torch.float32
        if (dt == torch.bfloat16 and os.environ.get("SINGA_PAIRED_STEM", "1") != "0"
                and PairedStemConv.applies(x.data, self.W.shape) and not self.bias
                and self.kernel_size == (7, 7) and self.stride == (2, 2) and self.padding == (3, 3)
                and self.dilation == (1, 1) and self.group == 1):
            return PairedStemConv(bn_stats=getattr(self, "bn_stats", False))(x, self.W)
        return super().forward(InputPrep(dt)(x))


def _dual_bn_add_relu(bn: layer.BatchNorm2d, x, bn2: layer.BatchNorm2d, x2):
    """relu(bn(x) + bn2(x2)) -- fused (DualBNAddReLU) on the native path,
    else the two BN layers with the residual add.  SINGA_FUSED_DOWN_BN=0
    disables the fusion."""
    if (os.environ.get("SINGA_FUSED_DOWN_BN", "1") != "0" and not autograd._TRACE
            and F.dual_bn_add_relu_ok(x.data, x2.data)):
        for b, t in ((bn2, x2), (bn, x)):
            if not b._initialized:
                b.initialize(t)
                b._initialized = True
        return autograd.DualBNAddReLU(bn, bn2)(x, bn.scale, bn.bias, x2, bn2.scale, bn2.bias)
    res = bn2(x2)
    return bn(x, relu=True, residual=res)


def _feeds_bn(*convs):
    """Mark convolutions whose output goes straight into a BatchNorm: their
    epilogue sums the BN statistics (no separate statistics pass)."""
    for c in convs:
        c.bn_stats = True


class Bottleneck(layer.Layer):
    expansion = 4

    def __init__(self, planes: int, stride: int = 1, downsample: bool = False):
        super().__init__()
        self.conv1 = layer.Conv2d(planes, 1, bias=False)
        self.bn1 = layer.BatchNorm2d()
        self.conv2 = layer.Conv2d(planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = layer.BatchNorm2d()
        self.conv3 = layer.Conv2d(planes * self.expansion, 1, bias=False)
        self.bn3 = layer.BatchNorm2d()
        self.has_down = downsample
        if downsample:
            self.down_conv = layer.Conv2d(planes * self.expansion, 1, stride=stride, bias=False)
            self.down_bn = layer.BatchNorm2d()
        _feeds_bn(self.conv1, self.conv2, self.conv3, *([self.down_conv] if downsample else []))

    def forward(self, x):
        out = self.bn1(self.conv1(x), relu=True)
        # a fused residual tail below reads bn2's output column sums (summed in its apply pass)
        tail = autograd.training and F.BNRES and x.data.is_cuda and not autograd._TRACE
        out = self.bn2(self.conv2(out), relu=True, colsum=tail)
        c3 = self.conv3
        if self.has_down:
            dc = self.down_conv
            if (tail and os.environ.get("SINGA_FUSED_DOWN_TAIL", "1") != "0" and c3.kernel_size == (1, 1) and c3.stride == (1, 1) and tuple(c3.padding) == (0, 0)
                    and not c3.bias and c3.group == 1 and dc.kernel_size == (1, 1) and tuple(dc.padding) == (0, 0)
                    and dc.stride[0] == dc.stride[1] and not dc.bias and dc.group == 1
                    and F.bnres_ok(out.data, (c3.nb_kernels, out.shape[1], 1, 1), None, down=(x.data, dc.stride[0]))):
                # both branches of the tail as one operator with the algebraic
                # backward (ConvBNDualAddReLU): no pass over either conv output
                # (initialised in the unfused path's order: the same parameter-init draws)
                k4 = SimpleNamespace(shape=(1, c3.nb_kernels), device=x.device)  # what a BN's initialize reads
                for lyr, t in ((dc, x), (c3, out), (self.down_bn, k4), (self.bn3, k4)):
                    if not lyr._initialized:
                        lyr.initialize(t)
                        lyr._initialized = True
                b3, bd = self.bn3, self.down_bn
                return autograd.ConvBNDualAddReLU(b3, bd, dc.stride[0])(out, c3.W, b3.scale, b3.bias, x, dc.W,
                                                                        bd.scale, bd.bias)
            xd = self.down_conv(x)  # (creation order as before the fusion: same parameter-init draws)
            return _dual_bn_add_relu(self.bn3, self.conv3(out), self.down_bn, xd)
        if (autograd.training and not autograd._TRACE and c3.kernel_size == (1, 1) and c3.stride == (1, 1)
                and tuple(c3.padding) == (0, 0) and not c3.bias and c3.group == 1
                and F.bnres_ok(out.data, (c3.nb_kernels, out.shape[1], 1, 1), x.data)):
            # the residual tail as one operator: its backward runs algebraically
            # (F.bnres_bwd) -- no pass over conv3's output or its gradient
            for lyr, t in ((c3, out), (self.bn3, x)):
                if not lyr._initialized:
                    lyr.initialize(t)
                    lyr._initialized = True
            bn = self.bn3
            return autograd.ConvBNAddReLU(bn.running_mean.data, bn.running_var.data, 1.0 - bn.momentum,
                                          bn.eps)(out, c3.W, bn.scale, bn.bias, x)
        return self.bn3(self.conv3(out), relu=True, residual=x)


class BasicBlock(layer.Layer):
    expansion = 1

    def __init__(self, planes: int, stride: int = 1, downsample: bool = False):
        super().__init__()
        self.conv1 = layer.Conv2d(planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = layer.BatchNorm2d()
        self.conv2 = layer.Conv2d(planes, 3, padding=1, bias=False)
        self.bn2 = layer.BatchNorm2d()
        self.has_down = downsample
        if downsample:
            self.down_conv = layer.Conv2d(planes, 1, stride=stride, bias=False)
            self.down_bn = layer.BatchNorm2d()
        _feeds_bn(self.conv1, self.conv2, *([self.down_conv] if downsample else []))

    def forward(self, x):
        out = self.bn1(self.conv1(x), relu=True)
        if self.has_down:
            xd = self.down_conv(x)
            return _dual_bn_add_relu(self.bn2, self.conv2(out), self.down_bn, xd)
        return self.bn2(self.conv2(out), relu=True, residual=x)


class ResNet(model.Model):
    def __init__(self, block, layers: Sequence[int], num_classes: int = 1000, num_channels: int = 3,
                 compute_dtype=torch.bfloat16):
        super().__init__()
        self.compute_dtype = compute_dtype
        self.num_classes = num_classes
        self.conv1 = StemConv2d(num_channels, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = layer.BatchNorm2d()
        _feeds_bn(self.conv1)
        self.maxpool = layer.MaxPool2d(3, 2, 1)
        blocks: List[layer.Layer] = []
        inplanes = 64
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
            stride = 1 if i == 0 else 2
            for j in range(n):
                s = stride if j == 0 else 1
                down = j == 0 and (s != 1 or inplanes != planes * block.expansion)
                blocks.append(block(planes, s, down))
                inplanes = planes * block.expansion
        self.blocks = blocks
        self.pool = layer.GlobalAvgPool2d()
        self.fc = layer.Linear(num_classes)
        self.loss_fn = layer.SoftMaxCrossEntropy()

    def forward(self, x):
        self.conv1.compute_dtype = self.compute_dtype
        x = self.conv1(x)  # the stem converts the fp32 NCHW batch itself
        mp = self.maxpool
        if (os.environ.get("SINGA_FUSED_STEM_POOL", "1") != "0" and not autograd._TRACE and mp.is_max
                and F.bn_relu_maxpool_ok(x.data, mp.kernel_size, mp.stride, mp.padding, mp.ceil_mode)):
            # BN + ReLU + max-pool in one pass (the 112x112x64 BN output is never written)
            bn = self.bn1
            if not bn._initialized:
                bn.initialize(x)
                bn._initialized = True
            x = autograd.BnReluMaxPool(bn.running_mean.data, bn.running_var.data, 1.0 - bn.momentum, bn.eps,
                                       mp.kernel_size, mp.stride, mp.padding)(x, bn.scale, bn.bias)
        else:
            x = self.maxpool(self.bn1(x, relu=True))
        for b in self.blocks:
            x = b(x)
        x = self.pool(x)
        return self.fc(x)

    def train_one_batch(self, x, y):
        out = self.forward(x)
        loss = self.loss_fn(out, y)
        self.optimizer(loss)
        return out, loss


def resnet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)


def create_model(depth: int = 50, **kw) -> ResNet:
    return {18: resnet18, 34: resnet34, 50: resnet50, 101: resnet101, 152: resnet152}[depth](**kw)
