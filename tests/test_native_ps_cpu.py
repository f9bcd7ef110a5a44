"""Native host runtime: C++ updaters (C13) and the native parameter server /
client (C25 / C26 / C12 / C15), CPU only."""
import json
import os
import threading

import numpy as np
import pytest
import torch

from singa_amd import _core as C
from singa_amd import opt
from singa_amd.parallel.ps import ParamServer, PSClient, PSSync

from test_tools_cpu import TINY, _run

KINDS = [("sgd", dict(momentum=0.9)), ("sgd", dict(momentum=0.9, nesterov=True)), ("sgd", dict(momentum=0.0)),
         ("sgd_ref", dict(momentum=0.9)), ("nesterov_ref", dict(momentum=0.9)), ("adagrad", {}), ("rmsprop", {}),
         ("adadelta", {}), ("adam", {}), ("adam", dict(adamw=True))]


@pytest.mark.parametrize("kind,kw", KINDS)
def test_native_updater_matches_reference_math(kind, kw):
    """C++ OptUpdate == the optimiser's reference math (Optimizer._cpu_update)
    over several steps, with per-element lr/wd multipliers and grad_scale."""
    rng = np.random.RandomState(0)
    n = 300001  # > one parallel_for grain: exercises the thread split
    o = opt.Optimizer(lr=0.05, weight_decay=1e-3, eps=1e-6, rho=0.9, **{k: v for k, v in kw.items()
                                                                          if k in ("momentum", "nesterov", "adamw")})
    o.kind = kind
    w0 = rng.randn(n).astype(np.float32)
    lr_vec = rng.uniform(0.5, 1.5, n).astype(np.float32)
    wd_vec = rng.uniform(0.0, 2.0, n).astype(np.float32)
    w_ref, s1_ref, s2_ref = torch.from_numpy(w0.copy()), torch.zeros(n), torch.zeros(n)
    w, s1, s2 = w0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for t in range(1, 4):
        g = rng.randn(n).astype(np.float32)
        o._cpu_update(w_ref, torch.from_numpy(g), s1_ref, s2_ref, torch.from_numpy(lr_vec) * 0.05,
                      torch.from_numpy(wd_vec) * 1e-3, float(t), 0.5)
        C.opt_update(C.updater_kind(kind), w, g, s1, s2, 0.05, 1e-3, 0.5, float(t), momentum=o.momentum,
                     eps=1e-6, rho=0.9, nesterov=o.nesterov, adamw=o.adamw, lr_vec=lr_vec, wd_vec=wd_vec)
    np.testing.assert_allclose(w, w_ref.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(s1, s1_ref.numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("method", ["kFixed", "kLinear", "kExponential", "kInverse_t", "kInverse", "kStep"])
def test_native_learning_rate_schedules(method):
    ref = opt.RefSchedule(method, 0.1, 0.01, 50, 0.5, 0.75)
    for step in (0, 1, 25, 49, 50, 51, 200):
        assert C.learning_rate(method, 0.1, 0.01, 50, 0.5, 0.75, step) == pytest.approx(ref(step), rel=1e-9)


@pytest.fixture
def servers():
    made = []

    def make(n=1, nworkers=1):
        for _ in range(n):
            made.append(ParamServer(0, nworkers))
        return made[-n:]
    yield make
    for s in made:
        s.close()


def test_ps_put_get_deferred_and_update(servers):
    (s,) = servers(1)
    cl = PSClient([f"127.0.0.1:{s.port}"])
    # a Get before the Put is deferred by the server until the key exists
    got = np.zeros(5, np.float32)
    th = threading.Thread(target=lambda: PSClient([f"127.0.0.1:{s.port}"]).get(3, got))
    th.start()
    threading.Event().wait(0.3)
    assert th.is_alive()
    cl.put(3, np.arange(5, dtype=np.float32))
    th.join(timeout=10)
    assert not th.is_alive() and np.array_equal(got, np.arange(5, dtype=np.float32))
    # server-side updater: reference SGD with momentum, h = m h + lr g; w -= h
    s.set_updater("sgd_ref", momentum=0.9, base_lr=0.1)
    w = np.zeros(5, np.float32)
    g = np.ones(5, np.float32)
    cl.update(3, g, w)
    np.testing.assert_allclose(w, np.arange(5) - 0.1, rtol=1e-6)
    cl.update(3, g, w)
    np.testing.assert_allclose(w, np.arange(5) - 0.1 - 0.19, rtol=1e-6)
    np.testing.assert_allclose(s.value(3), w)


def test_ps_elastic_and_random_sync_math(servers):
    (s,) = servers(1)
    cl = PSClient([f"127.0.0.1:{s.port}"])
    c0 = np.linspace(-1, 1, 11).astype(np.float32)
    cl.put(0, c0)
    w = (c0 + 1.0).astype(np.float32)
    cl.elastic(0, w, 0.25)  # d = 0.25 (w - c) = 0.25: c += d, w -= d
    np.testing.assert_allclose(s.value(0), c0 + 0.25, rtol=1e-6)
    np.testing.assert_allclose(w, c0 + 0.75, rtol=1e-6)
    # RandomSync: c[idx] += delta, reply old c[idx]; idx = (off + i*stride) % n
    off, stride, m = 3, 4, 6
    idx = (off + np.arange(m) * stride) % 11
    before = s.value(0)
    delta = np.arange(m, dtype=np.float32)
    old = np.zeros(m, np.float32)
    cl.random_sync(0, delta, old, off, stride)
    np.testing.assert_allclose(old, before[idx])
    after = before.copy()
    after[idx] += delta
    np.testing.assert_allclose(s.value(0), after)


def test_ps_pipelined_replace_collect_two_servers(servers):
    """pm benchmark pattern: Update (replace) every key, then Collect all
    replies; keys are sharded over 2 servers by id % 2."""
    ss = servers(2, nworkers=1)
    cl = PSClient([f"127.0.0.1:{s.port}" for s in ss])
    shapes = [(784 * 25,), (250,), (2000,), (10,)]
    for k, sh in enumerate(shapes):
        cl.put(k, np.zeros(sh, np.float32))
    vals = [np.full(sh, k + 1, np.float32) for k, sh in enumerate(shapes)]
    for k, v in enumerate(vals):
        cl.push_replace(k, v)
    outs = [np.zeros(sh, np.float32) for sh in shapes]
    assert cl.collect(list(range(len(shapes))), outs) == len(shapes)
    for k, o in enumerate(outs):
        assert np.all(o == k + 1)
        assert np.all(ss[k % 2].value(k) == k + 1)  # P7 key sharding
    cl.stop()
    assert ss[0].wait_stop(5.0) and ss[1].wait_stop(5.0)


def test_ps_sync_two_groups_easgd(servers):
    """Two worker groups exchanging through the native PS: group 1 bootstraps
    from group 0's Put; an elastic exchange moves both towards the centre."""
    from singa_amd.tensor import Tensor

    (s,) = servers(1, nworkers=2)
    ep = [f"127.0.0.1:{s.port}"]

    def store_for(v):
        ps = [Tensor(data=torch.full((4, 3), v)), Tensor(data=torch.full((7,), v))]
        for p in ps:
            p.requires_grad = p.stores_grad = True
        return opt.SGD(0.1).attach(ps)

    st0, st1 = store_for(1.0), store_for(5.0)
    sy0 = PSSync(st0, PSClient(ep), 0, 2, moving_rate=0.5)
    sy1 = PSSync(st1, PSClient(ep), 1, 2, moving_rate=0.5)
    sy0.bootstrap()
    sy1.bootstrap()
    assert all(torch.all(p.data == 1.0) for p in st1.params)  # group 1 received group 0's weights
    for p in st1.params:
        p.data.fill_(3.0)  # group 1 drifted: w1 = 3, centre = 1
    sy1.sync()
    # alpha = 0.5 / 2: d = 0.25 * (3 - 1) = 0.5 -> centre 1.5, w1 2.5
    assert all(torch.allclose(p.data, torch.full_like(p.data, 2.5)) for p in st1.params)
    assert np.allclose(s.value(0), 1.5) and np.allclose(s.value(1), 1.5)
    sy0.client.stop()
    sy1.client.stop()
    assert s.wait_stop(5.0)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("ptype", ["Elastic", "RandomSync"])
def test_launcher_two_workers_one_native_server(tmp_path, ptype):
    """The reference deployment: 2 worker groups + 1 parameter-server process
    (launch --nservers 1): the server Puts/serves, the workers sync every 2
    steps and send kStop; every process exits cleanly."""
    conf = tmp_path / "m.conf"
    conf.write_text((TINY % 6).replace("moving_rate: 0.5", f'moving_rate: 0.5 param_type: "{ptype}"'))
    port = 20000 + (os.getpid() * 7) % 20000
    cl = tmp_path / "c.conf"
    cl.write_text(f'nworkers: 2\nnservers: 1\nstart_port: {port}\nworkspace: "{tmp_path}/ws"\n')
    mj = tmp_path / "m.jsonl"
    r = _run(["-m", "singa_amd.launch", "--nproc", "2", "--nservers", "1", "--timeout", "240", "--",
              "--model_conf", str(conf), "--cluster_conf", str(cl), "--device", "cpu", "--synthetic",
              "--data_shape", "6,6", "--metrics_json", str(mj)], timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "[server 0] has shut down" in r.stderr
    losses = [json.loads(l)["loss"] for l in mj.read_text().splitlines()]
    assert len(losses) == 5 and all(np.isfinite(losses))  # steps 1-5 (step 0 is the local warm-up)


def test_ps_rejects_untrusted_requests(servers):
    """Server-side validation of values read off the socket: a RandomSync
    progression outside [0, n) or against an empty value, and a Replace that
    would change a key's size (its optimiser state keeps the Put's size), are
    rejected instead of indexing out of bounds; an oversized reply raises on
    the client instead of leaving the buffer silently unchanged."""
    (s,) = servers(1)
    cl = PSClient([f"127.0.0.1:{s.port}"])
    cl.put(0, np.arange(8, dtype=np.float32))
    old = np.zeros(3, np.float32)
    for a, b in ((-1, 1), (2, -3), (8, 1), (0, 9)):
        with pytest.raises(RuntimeError, match="rejected"):
            cl.random_sync(0, np.ones(3, np.float32), old, a, b)
    cl.put(1, np.zeros(0, np.float32))
    with pytest.raises(RuntimeError, match="rejected"):
        cl.random_sync(1, np.ones(2, np.float32), np.zeros(2, np.float32), 0, 1)
    # a size-changing Replace is rejected; the value and its optimiser state keep their size
    cl.push_replace(0, np.ones(16, np.float32))
    with pytest.raises(RuntimeError, match="rejected"):
        cl.collect([0], [np.zeros(16, np.float32)])
    np.testing.assert_allclose(s.value(0), np.arange(8))
    s.set_updater("sgd_ref", momentum=0.9, base_lr=0.1)
    w = np.zeros(8, np.float32)
    cl.update(0, np.ones(8, np.float32), w)  # still the 8-float key: no overflow of s1
    np.testing.assert_allclose(w, np.arange(8) - 0.1, rtol=1e-6)
    # a reply larger than the caller's buffer is an error, not a silent no-op
    small = np.zeros(4, np.float32)
    with pytest.raises(RuntimeError, match="exceeds"):
        cl.get(0, small)
    # the connection stays usable (the payload was drained)
    full = np.zeros(8, np.float32)
    assert cl.get(0, full) == 8
