"""VGG-11/13/16/19 (with optional BatchNorm) for 224x224 or 32x32 inputs."""
from __future__ import annotations

import torch

from .. import autograd, layer, model

CFGS = {11: [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
        13: [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
        16: [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
        19: [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]}


class VGG(model.Model):
    def __init__(self, depth: int = 16, num_classes: int = 1000, batch_norm: bool = True, small: bool = False,
                 compute_dtype=torch.bfloat16, num_channels: int = 3, dropout: float = 0.5):
        super().__init__()
        self.compute_dtype = compute_dtype
        self.convs, self.bns, self.kinds = [], [], []
        cin = num_channels  # explicit: the GPU input is channel-padded to 8, the weights are not
        for v in CFGS[depth]:
            if v == "M":
                self.kinds.append("M")
                self.convs.append(layer.MaxPool2d(2, 2))
                self.bns.append(None)
            else:
                self.kinds.append("C")
                self.convs.append(layer.Conv2d(cin, v, 3, padding=1, bias=not batch_norm,
                                               activation="NOTSET" if batch_norm else "RELU"))
                cin = v
                self.bns.append(layer.BatchNorm2d() if batch_norm else None)
        hid = 512 if small else 4096
        self.fc1, self.fc2 = layer.Linear(hid), layer.Linear(hid)
        self.r1, self.r2 = layer.ReLU(), layer.ReLU()
        self.d1, self.d2 = layer.Dropout(dropout), layer.Dropout(dropout)
        self.fc3 = layer.Linear(num_classes)
        self.loss_fn = layer.SoftMaxCrossEntropy()

    def forward(self, x):
        if x.data.is_cuda and x.dtype != self.compute_dtype:
            from .resnet import InputPrep

            x = InputPrep(self.compute_dtype)(x)
        for k, c, bn in zip(self.kinds, self.convs, self.bns):
            x = c(x)
            if bn is not None:
                x = bn(x, relu=True)
        x = autograd.flatten(x, 1)
        x = self.d1(self.r1(self.fc1(x)))
        x = self.d2(self.r2(self.fc2(x)))
        return self.fc3(x)

    def train_one_batch(self, x, y):
        out = self.forward(x)
        loss = self.loss_fn(out, y)
        self.optimizer(loss)
        return out, loss


def create_model(depth=16, **kw) -> VGG:
    return VGG(depth, **kw)
