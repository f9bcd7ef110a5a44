"""Micro-batched pipeline execution of a placed net (reference P6: layers
placed on several locations, BridgeSrc/BridgeDst hand-offs,
src/worker/worker.cc:136-155,216-302).

The reference ran a placed net one whole batch at a time: while location 1
computed, location 0 idled.  Here a training step splits the batch into
``m`` micro-batches and runs them through the stages on a pipeline
schedule, so the stages overlap:

* ``gpipe`` -- every micro-batch forward, then every backward (in reverse
  order); activations of all m micro-batches are alive at the peak;
* ``1f1b``  -- stage s runs ``S - s - 1`` warm-up forwards, then alternates
  one forward / one backward, then drains the remaining backwards: at most
  ``S - s`` micro-batches in flight per stage (PipeDream-flush order).

Both schedules accumulate the parameter gradients of the m micro-batches in
the flat gradient store (every backward kernel accumulates), with each
loss scaled by 1/m: the step's gradient equals the full-batch gradient of
the mean loss, so a pipelined placed net trains exactly like the unplaced
one (up to float summation order).  Normalisation layers see micro-batch
statistics (the usual GPipe caveat).

Across processes the stages exchange activations / gradients through the
bridge operators (non-blocking sends, blocking receives, one ordered
channel per direction); the schedules keep every process's sends and
receives in matching order, so no stage can deadlock.  In one process
(several locations = several devices) both schedules are valid orders of
the same work.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from .. import memory as _mem
from .. import autograd

SCHEDULES = ("gpipe", "1f1b")


def stage_of(net) -> Tuple[int, int]:
    """(this process's stage, number of stages).  Locations map to group
    ranks ``loc % world``; the stage order is the group-rank order."""
    if not getattr(net, "dist", False):
        return 0, 1
    return net.comm.rank, net.comm.world_size


def schedule(kind: str, m: int, stage: int, stages: int) -> List[Tuple[str, int]]:
    """The ordered list of ("F" | "B", micro-batch) actions of one stage."""
    if kind == "gpipe":
        return [("F", i) for i in range(m)] + [("B", i) for i in reversed(range(m))]
    if kind != "1f1b":
        raise ValueError(f"unknown pipeline schedule {kind!r} (use one of {SCHEDULES})")
    warm = min(stages - stage - 1, m)
    acts = [("F", i) for i in range(warm)]
    f, b = warm, 0
    while f < m:
        acts.append(("F", f))
        f += 1
        acts.append(("B", b))
        b += 1
    acts += [("B", i) for i in range(b, m)]
    return acts


def pipelined_step(net, zero_grad, m: int, kind: str = "1f1b") -> np.ndarray:
    """Forward + backward of one batch of ``net`` as ``m`` micro-batches on
    schedule ``kind``; gradients accumulate into the parameters' gradient
    store (``zero_grad`` clears it first).  Returns the step's metrics
    [loss, precision] averaged over the micro-batches (group-reduced)."""
    if m < 1:
        raise ValueError("micro-batches must be >= 1")
    stage, stages = stage_of(net)
    losses = net.loss_layers()
    saved = [l.loss_scale for l in losses]
    for l in losses:
        l.loss_scale = (l.loss_scale or 1.0) / m  # mean over the whole batch
    roots = {}
    met = np.zeros(2, np.float64)
    zero_grad()
    acts = schedule(kind, m, stage, stages)
    try:
        for n, (act, i) in enumerate(acts):
            if act == "F":
                outs = net.forward(training=True, micro=(i, m))
                roots[i] = net.backward_roots(outs)
                met += net.metrics(reduce=False)
            else:
                rs, seeds = roots.pop(i)
                autograd.training = True
                if rs:
                    for _ in autograd.backward(rs, seeds):
                        pass
            # Sends are deferred so that a send crossing a peer's send (1F1B's
            # steady state: activation i+1 downstream while gradient j comes
            # up) is grouped with the receive that matches it.  Between two
            # actions of the same kind no peer sends towards this process
            # (forwards only receive from upstream / send downstream; a
            # downstream stage in its drain sends gradients only after all
            # this stage's activations have arrived), so the deferred sends
            # leave right away: the next stage starts on micro-batch i while
            # this one computes i+1 (GPipe's and the warm-up / drain overlap).
            ch = getattr(net, "_pending", None)
            if ch is not None and hasattr(ch, "flush") and n + 1 < len(acts) and acts[n + 1][0] == act:
                ch.flush()
        net.finish_step()
    finally:
        for l, s in zip(losses, saved):
            l.loss_scale = s
        autograd.training = False
    # metric blobs above were scaled by the per-micro loss_scale (1/m): their
    # sum is the batch mean; reduce over the group once, outside the schedule
    if getattr(net, "dist", False):
        import torch

        from ..ops import glue as G
        t = G.copy_(_mem.empty(2, dtype=torch.float32, device=net.dev.torch_device),
                    torch.tensor(met, dtype=torch.float32))
        net.comm.all_reduce(t)
        met = t.cpu().double().numpy()
    return met
