"""Bridge operators: activations/gradients across locations (reference P6,
BridgeSrc/BridgeDst layers + the executor's ZeroMQ PUSH/PULL hand-off,
src/worker/worker.cc:216-299, include/worker/base_layer.h:264-312).

* :class:`ToDevice` -- one process driving several devices: a copy on the
  destination's stream; the gradient is copied back in backward.
* :class:`BridgeSend` / :class:`BridgeRecv` -- locations owned by different
  processes (one GPU each): p2p send/recv over RCCL (xGMI) or gloo.  Every
  payload is preceded by a small int64 header so the
  receiver can rebuild the tensor (dtype, requires-grad flag, shape).

Deadlock freedom: every process executes its local layers in the same global
topological order (sends are non-blocking, receives block), and the autograd
engine runs ready operators in decreasing forward order
(:func:`singa_amd.autograd.backward`), so a blocking gradient receive in
``BridgeSend.backward`` only ever waits for work at strictly later positions
of the global order -- which no process can be blocked on.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from .. import autograd
from ..autograd import Operator, _next_seq
from ..tensor import Tensor
from ..ops import glue as G

_MAXD = 8
_DT = [torch.float32, torch.bfloat16, torch.float16, torch.int32, torch.int64, torch.uint8]


def _code(dt: torch.dtype) -> int:
    return _DT.index(dt) if dt in _DT else 0


class ToDevice(Operator):
    def __init__(self, dev, name=None):
        super().__init__(name)
        self.dev = dev

    def forward(self, x):
        self.src_dev = x.device
        return x.to(self.dev.torch_device, non_blocking=True)

    def backward(self, dy):
        return dy.to(self.src_dev, non_blocking=True)


def to_device(x: Tensor, dev) -> Tensor:
    if x.data.device == dev.torch_device:
        return x
    if x.requires_grad and autograd.training:
        y = ToDevice(dev)(x)
        y.device = dev
        return y
    return Tensor(device=dev, data=x.data.to(dev.torch_device), requires_grad=False)


class BridgeSend(Operator):
    """Forward: isend x to ``peer``.  Backward: blocking recv of dL/dx."""

    always_run = True

    def __init__(self, comm, peer: int, pending: List, name=None):
        super().__init__(name)
        self.comm, self.peer, self.pending = comm, peer, pending

    def forward(self, x):
        if x.dim() > _MAXD:
            raise ValueError(f"bridge payloads support at most {_MAXD} dims")
        shp = list(x.shape) + [0] * (_MAXD - x.dim())
        hdr = torch.tensor([_code(x.dtype), int(self.requires_grad), x.dim()] + shp, dtype=torch.int64)
        payload = G.contiguous(x)
        dev_hdr = hdr.to(x.device)
        self.pending.append((self.comm.isend(dev_hdr, self.peer), dev_hdr))
        self.pending.append((self.comm.isend(payload, self.peer), payload))
        if self.requires_grad:
            self.shape, self.dtype, self.device = x.shape, x.dtype, x.device
        return x

    def backward(self, dy=None):
        g = torch.empty(self.shape, dtype=self.dtype, device=self.device)
        self.comm.recv(g, self.peer)
        return g


def bridge_send(x: Tensor, comm, peer: int, pending: List) -> Optional[Tensor]:
    """Returns the root tensor to include in backward (None if no grad)."""
    op = BridgeSend(comm, peer, pending)
    y = op(x)
    return y if op.requires_grad else None


class BridgeRecv(Operator):
    """Forward: blocking recv from ``peer``.  Backward: isend dL/dy (zeros
    if nothing downstream produced a gradient)."""

    always_run = True

    def __init__(self, comm, peer: int, pending: List, name=None):
        super().__init__(name)
        self.comm, self.peer, self.pending = comm, peer, pending

    def __call__(self, dev) -> Tensor:
        hdr = torch.empty(3 + _MAXD, dtype=torch.int64, device=dev.torch_device)
        self.comm.recv(hdr, self.peer)
        h = [int(v) for v in hdr.cpu().tolist()]
        code, rg, nd = h[0], h[1], h[2]
        shape = h[3:3 + nd]
        dt = _DT[code]
        buf = torch.empty(tuple(shape), dtype=dt, device=dev.torch_device)
        self.comm.recv(buf, self.peer)
        self.requires_grad = bool(rg) and autograd.training
        if not self.requires_grad:
            return Tensor(device=dev, data=buf, requires_grad=False)
        self.src, self.src_idx, self.params, self.input_requires = [], [], [], []
        self.shape, self.dtype, self.dev = buf.shape, buf.dtype, dev
        y = Tensor(device=dev, data=buf, requires_grad=True, creator=self)
        self.n_out = 1
        self._yid = {id(y): 0}
        self._seq = _next_seq()
        return y

    def backward(self, dy=None):
        if dy is None:
            dy = G.zeros(self.shape, self.dtype, self.dev.torch_device)
        dy = G.contiguous(G.to(dy, self.dtype))
        self.pending.append((self.comm.isend(dy, self.peer), dy))
        return ()


def wait_all(pending: List) -> None:
    for h, _ in pending:
        if h is not None:
            h.wait()
    pending.clear()
