"""LeNet-style CNN (reference examples/mnist/conv.conf: conv 20@5x5 -> max-pool
2/2 -> conv 50@5x5 -> max-pool 2/2 -> fc 500 -> ReLU -> fc 10)."""
from __future__ import annotations

from .. import autograd, layer, model


class CNN(model.Model):
    def __init__(self, num_classes: int = 10, num_channels: int = 1, conv1: int = 20, conv2: int = 50,
                 fc: int = 500):
        super().__init__()
        self.num_channels = num_channels
        self.conv1 = layer.Conv2d(num_channels, conv1, 5)
        self.pool1 = layer.MaxPool2d(2, 2)
        self.conv2 = layer.Conv2d(conv1, conv2, 5)
        self.pool2 = layer.MaxPool2d(2, 2)
        self.fc1 = layer.Linear(fc)
        self.relu = layer.ReLU()
        self.fc2 = layer.Linear(num_classes)
        self.loss_fn = layer.SoftMaxCrossEntropy()

    def forward(self, x):
        if len(x.shape) == 3:
            x = autograd.reshape(x, (x.shape[0], 1, x.shape[1], x.shape[2]))
        y = self.pool1(self.conv1(x))
        y = self.pool2(self.conv2(y))
        y = autograd.flatten(y, 1)
        return self.fc2(self.relu(self.fc1(y)))

    def train_one_batch(self, x, y):
        out = self.forward(x)
        loss = self.loss_fn(out, y)
        self.optimizer(loss)
        return out, loss


def create_model(**kw) -> CNN:
    return CNN(**kw)
