"""In-process fake communicator (threads over shared memory) and fault
injection.  The same rank functions that the gloo
multi-process tests run are driven through :mod:`singa_amd.parallel.fake`,
so the two backends are held to one oracle."""
import time

import numpy as np
import pytest
import torch

from singa_amd.parallel.fake import CommTimeout, FaultPlan, RankKilled, run_threads
from test_distributed_cpu import _collectives, _data, _dp_rank, _easgd_rank, _mlp_model, _train

pytestmark = pytest.mark.timeout(300)


def test_fake_collectives_match_gloo_semantics():
    world = 2
    res = run_threads(_collectives, world)
    for r, o in enumerate(res):
        assert o["all_reduce"] == [world * i + 100 * sum(range(world)) for i in range(8)]
        assert o["broadcast"] == [2.0] * 4
        full = [sum(i * (k + 1) for k in range(world)) for i in range(world * 3)]
        assert o["reduce_scatter"] == full[r * 3:(r + 1) * 3]
        assert o["all_gather"] == [float(k) for k in range(world) for _ in range(2)]
        assert o["all_to_all"] == [10.0 * s + r for s in range(world)]
    assert res[1]["recv"] == [42.0, 43.0]


def test_fake_collectives_four_ranks():
    def fn(rank, world, comm):
        t = torch.full((3,), float(rank))
        comm.all_reduce(t, op="max")
        ag = torch.empty(world)
        comm.all_gather(ag, torch.tensor([float(rank)]))
        a2a = torch.empty(world)
        comm.all_to_all(a2a, torch.tensor([10.0 * rank + j for j in range(world)]))
        return t.tolist(), ag.tolist(), a2a.tolist()

    for r, (mx, ag, a2a) in enumerate(run_threads(fn, 4)):
        assert mx == [3.0] * 3 and ag == [0.0, 1.0, 2.0, 3.0]
        assert a2a == [10.0 * s + r for s in range(4)]


def test_fake_split_subgroups():
    def fn(rank, world, comm):
        even = comm.split([0, 2])
        odd = comm.split([1, 3])
        sub = even if rank % 2 == 0 else odd
        assert (even is None) == (rank % 2 == 1)
        t = torch.tensor([float(rank)])
        sub.all_reduce(t)
        return t.item(), sub.rank, sub.world_size

    res = run_threads(fn, 4)
    assert [r[0] for r in res] == [2.0, 4.0, 2.0, 4.0]
    assert [r[1] for r in res] == [0, 0, 1, 1]


def test_distopt_over_fake_equals_single_process():
    from singa_amd import opt

    X, Y = _data()
    ref, _ = _train(_mlp_model(), X, Y, 4, opt.SGD(0.1, 0.9, weight_decay=1e-4))
    res = run_threads(_dp_rank, 2, "sync", 0.001)
    for r in range(2):
        for k, v in ref.items():
            np.testing.assert_allclose(res[r][k], v, rtol=1e-4, atol=1e-5, err_msg=f"rank {r} {k}")


@pytest.mark.parametrize("sharded", [False, True])
def test_easgd_over_fake(sharded):
    res = run_threads(_easgd_rank, 2, sharded)
    c0, alpha = res[0][0], res[0][4]
    ds = [alpha * (wb - c0) for _, wb, _, _, _ in res]
    for r, (_, wb, wa, c, _) in enumerate(res):
        np.testing.assert_allclose(wa, wb - ds[r], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(c, c0 + ds[0] + ds[1], rtol=1e-6, atol=1e-6)


def _loop(rank, world, comm, n):
    t = torch.ones(4)
    for _ in range(n):
        comm.all_reduce(t)
        t.div_(world)
    return t.tolist()


def test_straggler_delay_keeps_results():
    plan = FaultPlan().delay(1, "all_reduce", 0.02)
    t0 = time.monotonic()
    res = run_threads(_loop, 3, 5, faults=plan)
    assert time.monotonic() - t0 >= 0.1
    assert all(r == [1.0] * 4 for r in res)
    assert sum(1 for e in plan.log if e[0] == "delay") == 5


def test_killed_rank_times_out_peers():
    plan = FaultPlan().kill(2, "all_reduce", nth=3)
    res = run_threads(_loop, 3, 5, faults=plan, timeout_s=0.5, return_exceptions=True)
    assert isinstance(res[2], RankKilled)
    assert isinstance(res[0], CommTimeout) and isinstance(res[1], CommTimeout)
    assert "collective #2" in str(res[0])  # the 3rd collective is the one that never completed


def test_dropped_message_detected():
    plan = FaultPlan().drop(0, "all_reduce", nth=2)
    res = run_threads(_loop, 2, 3, faults=plan, timeout_s=0.5, return_exceptions=True)
    assert all(isinstance(r, CommTimeout) for r in res)


def test_dropped_send_times_out_receiver():
    def fn(rank, world, comm):
        if rank == 0:
            comm.send(torch.ones(2), 1)
            return "sent"
        t = torch.empty(2)
        comm.recv(t, 0)
        return t.tolist()

    res = run_threads(fn, 2, faults=FaultPlan().drop(0, "send", 1), timeout_s=0.3, return_exceptions=True)
    assert res[0] == "sent" and isinstance(res[1], CommTimeout)
    assert run_threads(fn, 2)[1] == [1.0, 1.0]


def test_dead_ranks_reports_killed():
    plan = FaultPlan().kill(1, "barrier", 1)

    def fn(rank, world, comm):
        try:
            comm.barrier()
        except (CommTimeout, RankKilled):
            pass
        return comm.dead_ranks()

    assert run_threads(fn, 2, faults=plan, timeout_s=0.3) == [[1], [1]]


@pytest.mark.parametrize("ptype", ["Elastic", "RandomSync"])
def test_worker_two_groups_over_fake_with_straggler(ptype):
    """The config-driven Worker (two EASGD / RandomSync groups) on the fake
    backend, with group 1 a straggler on every collective: training still
    converges and both groups sync the same number of times."""
    from test_distributed_cpu import _worker_rank

    plan = FaultPlan().delay(1, "*", 0.002)
    res = run_threads(_worker_rank, 2, ptype, faults=plan, timeout_s=30)
    for losses, nsync, _ in res:
        assert nsync >= 10
        assert losses[-1] < losses[0]
    assert res[0][1] == res[1][1]
