"""Metrics (SINGA ``singa.metric``; the reference LossLayer kept
[loss, top-k precision], src/worker/layer.cc:718-752)."""
from __future__ import annotations

import numpy as np
import torch


def _np(x):
    if hasattr(x, "data") and isinstance(getattr(x, "data"), torch.Tensor):
        x = x.data
    if isinstance(x, torch.Tensor):
        return x.detach().float().cpu().numpy()
    return np.asarray(x)


class Metric:
    def forward(self, x, y):
        raise NotImplementedError

    def evaluate(self, x, y) -> float:
        return float(np.mean(self.forward(x, y)))


class Accuracy(Metric):
    """Top-k accuracy per sample (1 if the label is among the k largest)."""

    def __init__(self, top_k: int = 1):
        self.k = top_k

    def forward(self, x, y):
        p, t = _np(x), _np(y).astype(np.int64).reshape(-1)
        topk = np.argsort(-p, axis=1)[:, :self.k]
        return (topk == t[:, None]).any(axis=1).astype(np.float32)


class Precision(Metric):
    """Macro precision of the arg-max prediction over the classes present."""

    def forward(self, x, y):
        pred, t = _np(x).argmax(1), _np(y).astype(np.int64).reshape(-1)
        out = []
        for c in np.unique(pred):
            m = pred == c
            out.append(float((t[m] == c).mean()))
        return np.asarray(out or [0.0], np.float32)


class Recall(Metric):
    def forward(self, x, y):
        pred, t = _np(x).argmax(1), _np(y).astype(np.int64).reshape(-1)
        out = []
        for c in np.unique(t):
            m = t == c
            out.append(float((pred[m] == c).mean()))
        return np.asarray(out or [0.0], np.float32)


class MeanLoss(Metric):
    def forward(self, x, y=None):
        return _np(x).reshape(-1)
