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

from typing import List, Sequence

import torch

from .. import autograd, layer, model
from ..ops import functional as F
from ..ops import native as N
from ..tensor import Tensor


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
                y = torch.empty((x.shape[0], cp, x.shape[2], x.shape[3]), dtype=torch.bfloat16, device=x.device,
                                memory_format=torch.channels_last)
                N.lib().nchw_to_nhwc_pad(x.data_ptr(), y.data_ptr(), x.shape[0], C, x.shape[2], x.shape[3], cp,
                                         N.stream())
                return y
            return F.to_nhwc_bf16(x, cp) if self.dtype == torch.bfloat16 else x.to(
                memory_format=torch.channels_last)
        return x.to(self.dtype) if x.dtype != self.dtype else x

    def backward(self, dy):
        return None


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
        out = self.bn2(self.conv2(out), relu=True)
        res = self.down_bn(self.down_conv(x)) if self.has_down else x
        return self.bn3(self.conv3(out), relu=True, residual=res)


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
        res = self.down_bn(self.down_conv(x)) if self.has_down else x
        return self.bn2(self.conv2(out), relu=True, residual=res)


class ResNet(model.Model):
    def __init__(self, block, layers: Sequence[int], num_classes: int = 1000, num_channels: int = 3,
                 compute_dtype=torch.bfloat16):
        super().__init__()
        self.compute_dtype = compute_dtype
        self.num_classes = num_classes
        self.conv1 = layer.Conv2d(num_channels, 64, 7, stride=2, padding=3, bias=False)
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
        dt = self.compute_dtype if x.data.is_cuda else torch.float32
        x = InputPrep(dt)(x)
        x = self.bn1(self.conv1(x), relu=True)
        x = self.maxpool(x)
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
