"""AlexNet (Krizhevsky 2012 single-tower layout, 224x224 input): conv
11x11/4 -> LRN -> pool, conv 5x5 -> LRN -> pool, three 3x3 convs, pool, two
4096 FC with dropout, classifier.  Exercises every reference op family at
scale: LRN (F8/F9), dropout (F7), big FC GEMMs, max-pool, ReLU fused into
the conv epilogue.  A CIFAR-10-sized variant (``small=True``, 32x32 input)
follows the reference-era cuda-convnet layout."""
from __future__ import annotations

import torch

from .. import autograd, layer, model
from .resnet import InputPrep


class AlexNet(model.Model):
    def __init__(self, num_classes: int = 1000, num_channels: int = 3, small: bool = False, dropout: float = 0.5,
                 compute_dtype=torch.float32):
        super().__init__()
        self.small = small
        self.compute_dtype = compute_dtype
        if small:
            self.c1 = layer.Conv2d(num_channels, 32, 5, padding=2, activation="RELU")
            self.p1 = layer.MaxPool2d(3, 2)
            self.n1 = layer.LRN(3, 5e-5, 0.75, 1.0)
            self.c2 = layer.Conv2d(32, 32, 5, padding=2, activation="RELU")
            self.p2 = layer.AvgPool2d(3, 2)
            self.n2 = layer.LRN(3, 5e-5, 0.75, 1.0)
            self.c3 = layer.Conv2d(32, 64, 5, padding=2, activation="RELU")
            self.p3 = layer.AvgPool2d(3, 2)
            self.fcs = []
            self.drops = []
        else:
            self.c1 = layer.Conv2d(num_channels, 96, 11, stride=4, padding=2, activation="RELU")
            self.n1 = layer.LRN(5, 1e-4, 0.75, 2.0)
            self.p1 = layer.MaxPool2d(3, 2)
            self.c2 = layer.Conv2d(96, 256, 5, padding=2, activation="RELU")
            self.n2 = layer.LRN(5, 1e-4, 0.75, 2.0)
            self.p2 = layer.MaxPool2d(3, 2)
            self.c3 = layer.Conv2d(256, 384, 3, padding=1, activation="RELU")
            self.c4 = layer.Conv2d(384, 384, 3, padding=1, activation="RELU")
            self.c5 = layer.Conv2d(384, 256, 3, padding=1, activation="RELU")
            self.p3 = layer.MaxPool2d(3, 2)
            self.fcs = [layer.Linear(4096), layer.Linear(4096)]
            self.relus = [layer.ReLU(), layer.ReLU()]
            self.drops = [layer.Dropout(dropout), layer.Dropout(dropout)] if dropout > 0 else []
        self.fc = layer.Linear(num_classes)
        self.loss_fn = layer.SoftMaxCrossEntropy()

    def forward(self, x):
        if (x.data.is_cuda and x.dtype == torch.float32 and self.compute_dtype == torch.bfloat16
                and x.data.dim() == 4 and x.data.is_contiguous()):
            # fp32 NCHW images -> bf16 NHWC with the channels padded to 8 in one
            # pass (the first conv takes the padded input as is), instead of a
            # cast pass followed by the conv's own layout pass
            x = InputPrep(torch.bfloat16)(x)
        elif x.data.is_cuda and x.dtype != self.compute_dtype:
            x = autograd.cast(x, self.compute_dtype)
        if self.small:
            y = self.n1(self.p1(self.c1(x)))
            y = self.n2(self.p2(self.c2(y)))
            y = self.p3(self.c3(y))
        else:
            y = self.p1(self.n1(self.c1(x)))
            y = self.p2(self.n2(self.c2(y)))
            y = self.p3(self.c5(self.c4(self.c3(y))))
        y = autograd.flatten(y, 1)
        for i, fc in enumerate(self.fcs):
            y = self.relus[i](fc(y))
            if self.drops:
                y = self.drops[i](y)
        return self.fc(y)

    def train_one_batch(self, x, y):
        out = self.forward(x)
        loss = self.loss_fn(out, y)
        self.optimizer(loss)
        return out, loss


def create_model(**kw) -> AlexNet:
    return AlexNet(**kw)
