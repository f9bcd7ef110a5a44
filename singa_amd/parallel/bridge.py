"""Bridge operators: activations/gradients across locations (reference P6,
BridgeSrc/BridgeDst layers + the executor's ZeroMQ PUSH/PULL hand-off,
src/worker/worker.cc:216-299, include/worker/base_layer.h:264-312).

* :class:`ToDevice` -- one process driving several devices: a copy on the
  destination's stream; the gradient is copied back in backward.
* :class:`BridgeSend` / :class:`BridgeRecv` -- locations owned by different
  processes (one GPU each): p2p send/recv over RCCL (xGMI) or gloo through a
  per-process :class:`P2PChannel` (deferred sends issued as one RCCL group
  with the next receive, headers checked once per step).

Deadlock freedom: every process executes its local layers in the same global
topological order (sends are deferred and issued before -- on RCCL grouped
with -- the next blocking receive), and the autograd engine runs ready
operators in decreasing forward order (:func:`singa_amd.autograd.backward`),
so a blocking gradient receive in ``BridgeSend.backward`` only ever waits for
work at strictly later positions of the global order -- which no process can
be blocked on.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from .. import memory as _mem
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


class P2PChannel:
    """The point-to-point traffic of one process's bridges for one step.

    * Sends are DEFERRED: a bridge posts (tensor, peer) here; the queue is
      issued together with the next blocking receive -- as ONE RCCL group
      (ncclGroupStart/End) on the native communicator, as non-blocking isends
      on torch.distributed -- or at the end of the step.  All traffic of a
      process therefore runs on one stream in one order, and the crossing
      sends of a 1F1B schedule (stage s sends activation i+1 while its peer
      sends gradient i) are paired with the receives that match them instead
      of blocking each other (an ungrouped RCCL send of a large message waits
      for its receiver).
    * Headers: every payload is preceded by a small int64 header (dtype,
      requires-grad flag, shape).  By default a receiver reads every header
      on the host before it posts the payload receive, so a sender may change
      a tensor's shape at any step (a partial last batch, a new sequence
      length).  With ``static_shapes=True`` (a pipeline whose message shapes
      are fixed: the config-driven NeuralNet, whose data layers always yield
      full batches) a receiver reads a header on the host only the first time
      it sees a channel slot (peer, k-th receive of the step); afterwards it
      posts header and payload receives together from the cached shape and
      checks all the step's headers with ONE device-to-host copy in
      :meth:`finish` -- no host synchronisation per message.  (A shape change
      under that promise is an error: RCCL has no way to abort a posted
      receive of the wrong size.)
    * :meth:`flush` issues the deferred sends as one group without a receive;
      the pipeline schedules call it between consecutive actions of the same
      kind, where no peer can be sending towards this process (see
      :func:`singa_amd.parallel.pipeline.pipelined_step`)."""

    def __init__(self, comm, static_shapes: bool = False):
        self.comm = comm
        self.static_shapes = bool(static_shapes)
        self.log: List[tuple] = []  # ("send" | "recv", peer) in issue order (schedule-overlap tests)
        self.native = hasattr(comm, "p2p_group") and getattr(comm, "backend", "") == "rccl"
        self.sends: List[Tuple[torch.Tensor, int]] = []
        self.handles: List[tuple] = []
        self.shapes: dict = {}   # (peer, k) -> header list
        self.checks: List[tuple] = []  # (device header, expected header list, slot)
        self.hdrs: dict = {}     # header list -> device tensor (sender side cache)
        self.k: dict = {}        # peer -> receives this step
        self.host_reads = 0      # headers read on the host (first use of a slot only)
        self.flushes = 0         # send groups issued without a receive (schedule overlap)
        self.checked = 0         # headers verified in bulk at step end

    # compatibility with the plain pending-list protocol
    def append(self, item) -> None:
        self.handles.append(item)

    def post(self, t: torch.Tensor, peer: int) -> None:
        self.sends.append((t, peer))

    def header(self, x: torch.Tensor, rg: bool) -> torch.Tensor:
        shp = list(x.shape) + [0] * (_MAXD - x.dim())
        h = (_code(x.dtype), int(rg), x.dim(), *shp)
        t = self.hdrs.get((h, x.device))
        if t is None:
            t = self.hdrs[(h, x.device)] = torch.tensor(list(h), dtype=torch.int64).to(x.device)
        return t

    def _issue_sends(self) -> None:
        for t, peer in self.sends:
            self.log.append(("send", peer))
            if self.native:
                self.comm.send(t, peer)
            else:
                self.handles.append((self.comm.isend(t, peer), t))
        self.sends = []

    def exchange(self, bufs: List[torch.Tensor], peer: int) -> None:
        """Issue the deferred sends, then receive ``bufs`` (in order) from
        ``peer`` -- one group on RCCL."""
        if self.native:
            with self.comm.p2p_group():
                self._issue_sends()
                for b in bufs:
                    self.comm.recv(b, peer)
        else:
            self._issue_sends()
            for b in bufs:
                self.comm.recv(b, peer)
        self.log.extend(("recv", peer) for _ in bufs)

    def recv_tensor(self, peer: int, dev) -> Tuple[torch.Tensor, bool]:
        """Receive the next (header, payload) pair from ``peer``: (tensor,
        requires-grad flag of the sender)."""
        k = self.k.get(peer, 0)
        self.k[peer] = k + 1
        hdr = _mem.empty(3 + _MAXD, dtype=torch.int64, device=dev.torch_device)
        h = self.shapes.get((peer, k)) if self.static_shapes else None
        if h is None:  # first time on this slot (or shapes may change): read the header on the host
            self.exchange([hdr], peer)
            self.host_reads += 1
            h = self.shapes[(peer, k)] = [int(v) for v in hdr.cpu().tolist()]
            buf = _mem.empty(tuple(h[3:3 + h[2]]), dtype=_DT[h[0]], device=dev.torch_device)
            self.exchange([buf], peer)
        else:
            buf = _mem.empty(tuple(h[3:3 + h[2]]), dtype=_DT[h[0]], device=dev.torch_device)
            self.exchange([hdr, buf], peer)
            self.checks.append((hdr, h, (peer, k)))
        return buf, bool(h[1])

    def flush(self) -> None:
        if not self.sends:
            return
        self.flushes += 1
        if self.native:
            with self.comm.p2p_group():
                self._issue_sends()
        else:
            self._issue_sends()

    def finish(self) -> None:
        """End of step: issue what is left, complete it, verify the headers
        that were not read on the host (one copy for all of them)."""
        self.flush()
        for h, _ in self.handles:
            if h is not None:
                h.wait()
        self.handles.clear()
        self.k.clear()
        if self.checks:
            got = torch.stack([c[0] for c in self.checks]).cpu().tolist()
            for (_, exp, slot), g in zip(self.checks, got):
                if [int(v) for v in g] != exp:
                    self.shapes.pop(slot, None)
                    self.checks.clear()
                    raise RuntimeError(f"bridge header mismatch on slot {slot}: got {g}, expected {exp} (the "
                                       "sender's tensor shape changed between steps)")
            self.checked += len(self.checks)
            self.checks.clear()


def _chan(pending) -> P2PChannel:
    if not isinstance(pending, P2PChannel):
        raise TypeError("bridges need a P2PChannel (parallel.bridge.P2PChannel(comm))")
    return pending


class BridgeSend(Operator):
    """Forward: post x (header + payload) to ``peer``.  Backward: receive
    dL/dx (grouped with the deferred sends)."""

    always_run = True

    def __init__(self, comm, peer: int, pending: "P2PChannel", name=None):
        super().__init__(name)
        self.comm, self.peer, self.chan = comm, peer, _chan(pending)

    def forward(self, x):
        if x.dim() > _MAXD:
            raise ValueError(f"bridge payloads support at most {_MAXD} dims")
        payload = G.contiguous(x)
        self.chan.post(self.chan.header(payload, self.requires_grad), self.peer)
        self.chan.post(payload, self.peer)
        if self.requires_grad:
            self.shape, self.dtype, self.device = x.shape, x.dtype, x.device
        return x

    def backward(self, dy=None):
        g = _mem.empty(self.shape, dtype=self.dtype, device=self.device)
        self.chan.exchange([g], self.peer)
        return g


def bridge_send(x: Tensor, comm, peer: int, pending: "P2PChannel") -> Optional[Tensor]:
    """Returns the root tensor to include in backward (None if no grad)."""
    op = BridgeSend(comm, peer, pending)
    y = op(x)
    return y if op.requires_grad else None


class BridgeRecv(Operator):
    """Forward: receive from ``peer``.  Backward: post dL/dy (zeros if
    nothing downstream produced a gradient)."""

    always_run = True

    def __init__(self, comm, peer: int, pending: "P2PChannel", name=None):
        super().__init__(name)
        self.comm, self.peer, self.chan = comm, peer, _chan(pending)

    def __call__(self, dev) -> Tensor:
        buf, rg = self.chan.recv_tensor(self.peer, dev)
        self.requires_grad = rg and autograd.training
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
        self.chan.post(dy, self.peer)
        return ()


def wait_all(pending) -> None:
    if isinstance(pending, P2PChannel):
        pending.finish()
        return
    for h, _ in pending:
        if h is not None:
            h.wait()
    pending.clear()
