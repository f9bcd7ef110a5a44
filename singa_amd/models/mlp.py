"""Multi-layer perceptrons.

* :func:`deep_big_simple` -- the reference's MNIST MLP
  (examples/mnist/mlp.conf: 784-2500-2000-1500-1000-500-10 with the scaled
  tanh ``1.7159*tanh(0.6667x)``, include/mshadow/cxxnet_op.h:77-81);
* :class:`MLP` -- generic ``in -> hidden... -> classes`` with ReLU (the
  BASELINE minimum slice is 784-512-10).
"""
from __future__ import annotations

from typing import Sequence

from .. import layer, model


class MLP(model.Model):
    def __init__(self, hidden: Sequence[int] = (512,), num_classes: int = 10, activation: str = "relu",
                 dropout: float = 0.0, fuse_activation: bool = True):
        super().__init__()
        # relu / sigmoid / tanh / stanh run in the GEMM epilogues (forward, and
        # backward inside the next layer's data-gradient GEMM)
        fused = fuse_activation and activation in ("relu", "sigmoid", "tanh", "stanh")
        self.fcs = [layer.Linear(h, activation=activation if fused else None) for h in hidden]
        act = {"relu": layer.ReLU, "tanh": layer.Tanh, "stanh": layer.STanh, "sigmoid": layer.Sigmoid,
               "gelu": layer.Gelu, "identity": layer.Identity}["identity" if fused else activation]
        self.acts = [act() for _ in hidden]
        self.drops = [layer.Dropout(dropout) for _ in hidden] if dropout > 0 else []
        self.out = layer.Linear(num_classes)
        self.loss_fn = layer.SoftMaxCrossEntropy()

    def forward(self, x):
        if len(x.shape) > 2:
            from .. import autograd

            x = autograd.flatten(x, 1)
        for i, (fc, a) in enumerate(zip(self.fcs, self.acts)):
            x = fc(x) if fc.activation is not None else a(fc(x))
            if self.drops:
                x = self.drops[i](x)
        return self.out(x)

    def train_one_batch(self, x, y):
        out = self.forward(x)
        loss = self.loss_fn(out, y)
        self.optimizer(loss)
        return out, loss


def deep_big_simple(num_classes: int = 10) -> MLP:
    return MLP((2500, 2000, 1500, 1000, 500), num_classes, activation="stanh")


def create_model(hidden=(512,), num_classes=10, **kw) -> MLP:
    return MLP(hidden, num_classes, **kw)
