"""SINGA 3.x ``singa.module`` compatibility: ``Module`` is :class:`singa_amd.model.Model`
(graph capture, compile, train_one_batch, save/load states)."""
from .model import Model

Module = Model

__all__ = ["Module", "Model"]
