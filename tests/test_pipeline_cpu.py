"""Micro-batched pipeline execution of placed nets (singa_amd/parallel/pipeline.py;
reference P6 bridges, src/worker/worker.cc:136-155,216-302).

A placed 2-location net trained with m micro-batches per step (GPipe and
1F1B schedules) must equal the unplaced net trained on whole batches:
same loss history, same parameters -- in one process (both locations
local) and across two gloo processes (one stage each)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from dist_util import run_ranks  # noqa: E402
from singa_amd.parallel import pipeline as P  # noqa: E402

NET = """
train_steps: 5
display_frequency: 1
updater { base_learning_rate: 0.05 type: kSGD momentum: 0.9 weight_decay: 0.0001 }
neuralnet {
  layer { name: "data" type: "kSyntheticData" data_param { batchsize: 8 } }
  layer { name: "mnist" type: "kMnistImage" srclayers: "data" mnist_param { norm_a: 255 norm_b: 0 } }
  layer { name: "label" type: "kLabel" srclayers: "data" }
  layer { name: "conv1" type: "kConvolution" srclayers: "mnist" convolution_param { num_filters: 4 kernel: 3 }
          param { name: "wc" init_method: kUniform low: -0.3 high: 0.3 }
          param { name: "bc" init_method: kUniform low: -0.1 high: 0.1 } }
  layer { name: "pool1" type: "kPooling" srclayers: "conv1" pooling_param { pool: MAX kernel: 2 stride: 2 } }
  layer { name: "fc1" type: "kInnerProduct" srclayers: "pool1" inner_product_param { num_output: 12 } %s
          param { name: "w1" init_method: kUniform low: -0.2 high: 0.2 }
          param { name: "b1" init_method: kUniform low: -0.1 high: 0.1 } }
  layer { name: "tanh1" type: "kTanh" srclayers: "fc1" %s }
  layer { name: "fc2" type: "kInnerProduct" srclayers: "tanh1" inner_product_param { num_output: 10 } %s
          param { name: "w2" init_method: kUniform low: -0.2 high: 0.2 }
          param { name: "b2" init_method: kUniform low: -0.1 high: 0.1 } }
  layer { name: "loss" type: "kSoftmaxLoss" srclayers: "fc2" srclayers: "label" %s }
}
"""
_OV = {"*": {"shape": (8, 8), "nclass": 10, "seed": 5}}


def _conf(placed: bool) -> str:
    loc = "locationid: 1" if placed else ""
    return NET % ((loc,) * 4)


def _fix_batch(w):
    for l in w.train_net.layers:
        if l.is_data and w.train_net.is_local(l):
            s = l.source
            img, lab = s.next()
            s.next = lambda: (img, lab)


def _params(w):
    out = {}
    for l in w.train_net.layers:
        if w.train_net.is_local(l):
            for p in l.params:
                out[p.name] = p.data.clone().numpy()
    return out


def _run_worker(placed, m=1, kind="1f1b", comm=None, cluster=None):
    from singa_amd.config import schema
    from singa_amd.runtime import Worker

    w = Worker(schema.parse_text("ModelProto", _conf(placed)), cluster, comm=comm, log=lambda s: None, seed=0,
               data_override=_OV, micro_batches=m, pipeline=kind)
    _fix_batch(w)
    w.run()
    return [float(h[2][0]) for h in w.history if h[0] == "train"], _params(w)


def _reference():
    from singa_amd.parallel import communicator

    communicator.reset()
    return _run_worker(False)


# ------------------------------------------------------------------ schedules
def _simulate(kind, m, S):
    """Run S stages' action lists with blocking receives; returns True if
    every stage finishes (no deadlock) and dependencies hold."""
    acts = [P.schedule(kind, m, s, S) for s in range(S)]
    done = [set() for _ in range(S)]
    pos = [0] * S
    progress = True
    while progress:
        progress = False
        for s in range(S):
            if pos[s] == len(acts[s]):
                continue
            a, i = acts[s][pos[s]]
            if a == "F":
                ok = s == 0 or ("F", i) in done[s - 1]
            else:
                ok = ("F", i) in done[s] and (s == S - 1 or ("B", i) in done[s + 1])
            if ok:
                done[s].add((a, i))
                pos[s] += 1
                progress = True
    return all(pos[s] == len(acts[s]) for s in range(S))


@pytest.mark.parametrize("kind", P.SCHEDULES)
@pytest.mark.parametrize("m,S", [(1, 2), (4, 2), (4, 4), (8, 3), (2, 5)])
def test_schedules_are_complete_and_deadlock_free(kind, m, S):
    for s in range(S):
        acts = P.schedule(kind, m, s, S)
        assert sorted(acts) == sorted([("F", i) for i in range(m)] + [("B", i) for i in range(m)])
        for i in range(m):
            assert acts.index(("F", i)) < acts.index(("B", i))
    assert _simulate(kind, m, S)


def test_1f1b_bounds_in_flight_micro_batches():
    S, m = 4, 8
    for s in range(S):
        live = peak = 0
        for a, _ in P.schedule("1f1b", m, s, S):
            live += 1 if a == "F" else -1
            peak = max(peak, live)
        assert peak == S - s  # GPipe would hold all m
    assert max(sum(1 for a, _ in P.schedule("gpipe", m, 0, S)[:m] if a == "F"), 0) == m


# ------------------------------------------------------------------ in-process
@pytest.mark.parametrize("kind", P.SCHEDULES)
@pytest.mark.parametrize("m", [2, 4])
def test_placed_net_in_process_pipelined_equals_unplaced(kind, m, monkeypatch):
    ref_loss, ref_params = _reference()
    calls = []
    orig = P.pipelined_step

    def spy(net, zg, mm, kk):
        calls.append((mm, kk, sorted({l.type_name for l in net.layers if "Bridge" in l.type_name})))
        return orig(net, zg, mm, kk)
    monkeypatch.setattr(P, "pipelined_step", spy)
    loss, params = _run_worker(True, m, kind)
    assert len(calls) == 5 and calls[0] == (m, kind, ["kBridgeDst", "kBridgeSrc"])
    assert ref_loss[-1] < ref_loss[0]
    np.testing.assert_allclose(loss, ref_loss, rtol=1e-5, atol=1e-6)
    assert params.keys() == ref_params.keys()
    for k in ref_params:
        np.testing.assert_allclose(params[k], ref_params[k], rtol=1e-5, atol=1e-6, err_msg=k)


def test_unplaced_micro_batching_equals_whole_batch():
    ref_loss, ref_params = _reference()
    loss, params = _run_worker(False, 4, "gpipe")
    np.testing.assert_allclose(loss, ref_loss, rtol=1e-5, atol=1e-6)
    for k in ref_params:
        np.testing.assert_allclose(params[k], ref_params[k], rtol=1e-5, atol=1e-6, err_msg=k)


# ------------------------------------------------------------------ two processes
def _stage_worker(rank, world, comm, m, kind):
    from singa_amd.config import schema

    cp = schema.new("ClusterProto")
    cp.nworkers, cp.nprocs_per_group, cp.workspace = world, world, ""
    return _run_worker(True, m, kind, comm=comm, cluster=cp)


@pytest.mark.parametrize("kind", P.SCHEDULES)
def test_placed_net_across_processes_pipelined_equals_unplaced(kind):
    ref_loss, ref_params = _reference()
    res = run_ranks(_stage_worker, 2, 4, kind)
    seen = {}
    for r in range(2):
        loss, params = res[r]
        np.testing.assert_allclose(loss, ref_loss, rtol=1e-5, atol=1e-6, err_msg=f"rank {r}")
        seen.update(params)
    assert seen.keys() == ref_params.keys()  # the two stages hold disjoint halves
    for k in ref_params:
        np.testing.assert_allclose(seen[k], ref_params[k], rtol=1e-5, atol=1e-6, err_msg=k)


# ------------------------------------------- loopback RCCL ranks (threads)
def _stage_worker_chan(rank, world, comm, m, kind):
    from singa_amd.config import schema
    from singa_amd.runtime import Worker

    cp = schema.new("ClusterProto")
    cp.nworkers, cp.nprocs_per_group, cp.workspace = world, world, ""
    w = Worker(schema.parse_text("ModelProto", _conf(True)), cp, comm=comm, log=lambda s: None, seed=0,
               data_override=_OV, micro_batches=m, pipeline=kind)
    _fix_batch(w)
    w.run()
    ch = w.train_net._pending
    return ([float(h[2][0]) for h in w.history if h[0] == "train"], _params(w), comm, ch.host_reads, ch.checked,
            ch.flushes)


@pytest.mark.parametrize("kind", P.SCHEDULES)
def test_placed_net_over_loopback_rccl_grouped_p2p(kind):
    """The same 2-stage placed net on the REAL RcclCommunicator over the
    native loopback communicator, whose ungrouped sends are rendezvous (an
    RCCL-style crossing 1F1B exchange deadlocks there): the bridges' grouped,
    deferred sends complete every schedule, equal the unplaced net, read
    headers on the host only on the first step, and leave between actions of
    the same kind (stage overlap, not held back to the next receive)."""
    from singa_amd.parallel.loop import run_ranks as loop_ranks

    ref_loss, ref_params = _reference()
    m = 4
    res = loop_ranks(_stage_worker_chan, 2, m, kind, timeout_s=30.0)
    seen = {}
    for r in range(2):
        loss, params, comm, host_reads, checked, flushes = res[r]
        np.testing.assert_allclose(loss, ref_loss, rtol=1e-5, atol=1e-6, err_msg=f"rank {r}")
        seen.update(params)
        assert comm.loopback and comm.stats["calls"] > 0
        # stage 1 receives 2 bridges x m headed tensors per step (pool1 -> fc1
        # activations and the labels): read on the host in step 1 only,
        # bulk-checked in the other 4 steps; stage 0 receives the gradients,
        # whose shapes it already knows (no headers)
        assert (host_reads, checked) == ((2 * m, 4 * 2 * m) if r == 1 else (0, 0))
        # schedule overlap: between two actions of the same kind the deferred
        # sends leave at once (GPipe: stage 0 after each of its first m-1
        # forwards, stage 1 after each of its first m-1 backwards; 1F1B: stage
        # 0's one warm-up forward), plus stage 1's last gradient at the step's
        # end; 5 steps
        want = {"gpipe": (5 * (m - 1), 5 * m), "1f1b": (5, 5)}[kind]
        assert flushes == want[r], (kind, r, flushes)
    for k in ref_params:
        np.testing.assert_allclose(seen[k], ref_params[k], rtol=1e-5, atol=1e-6, err_msg=k)
