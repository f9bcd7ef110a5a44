"""Native RCCL communicator (csrc/comm/rccl_comm.cpp, parallel/rccl.py) on
the MI355X: the bindings on a 1-rank communicator (every collective, async
comm-stream handles, HIP-graph capture of a collective), and -- when RCCL
admits two ranks on the one GPU of the test box -- real 2-rank collectives
and a data-parallel step compared with a single-process step."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from dist_util import run_ranks  # noqa: E402

pytestmark = pytest.mark.gpu


def _one_rank(gpu):
    from singa_amd.parallel.rccl import RcclCommunicator
    return RcclCommunicator(1, 0, 0, store=None)


def test_rccl_one_rank_bindings(gpu):
    from singa_amd.ops import native as N
    c = _one_rank(gpu)
    nc, s = c._c, torch.cuda.current_stream().cuda_stream
    assert nc.nranks == 1 and nc.rank == 0 and N.lib().rccl_version() > 0
    x = torch.arange(1000, dtype=torch.float32, device=gpu)
    y = torch.empty_like(x)
    nc.all_reduce(x.data_ptr(), y.data_ptr(), x.numel(), 0, 0, s)  # out-of-place sum over 1 rank = copy
    for dt, code in ((torch.bfloat16, 1), (torch.int64, 4), (torch.float64, 6)):
        xb = x.to(dt)
        nc.all_reduce(xb.data_ptr(), xb.data_ptr(), xb.numel(), code, 2, s)  # max, in place
        assert torch.equal(xb.cpu(), x.to(dt).cpu())
    z = torch.empty_like(x)
    nc.all_gather(x.data_ptr(), z.data_ptr(), x.numel(), 0, s)
    w = torch.empty_like(x)
    nc.reduce_scatter(x.data_ptr(), w.data_ptr(), x.numel(), 0, 0, s)
    b = torch.empty_like(x)
    nc.broadcast(x.data_ptr(), b.data_ptr(), x.numel(), 0, 0, s)
    a2a = torch.empty_like(x)
    nc.all_to_all(x.data_ptr(), a2a.data_ptr(), x.numel(), 0, s)
    torch.cuda.synchronize()
    for t in (y, z, w, b, a2a):
        assert torch.equal(t.cpu(), x.cpu())
    assert c.async_error() == ""


def test_rccl_async_work_and_graph_capture(gpu):
    """An async collective runs on the comm stream and joins back through an
    event; a collective captured into a HIP graph replays correctly."""
    c = _one_rank(gpu)
    nc = c._c
    x = torch.full((1 << 20,), 2.0, device=gpu)
    w = c._run(True, (x,), lambda s: nc.all_reduce(x.data_ptr(), x.data_ptr(), x.numel(), 0, 0, s))
    w.wait()
    torch.cuda.synchronize()
    assert w.is_completed() and float(x[0]) == 2.0
    src = torch.zeros(4096, device=gpu)
    dst = torch.zeros(4096, device=gpu)
    # warm the communicator outside capture, then capture fork -> all-reduce -> join
    c._run(False, (src,), lambda s: nc.all_reduce(src.data_ptr(), dst.data_ptr(), src.numel(), 0, 0, s))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        wk = c._run(True, (src, dst), lambda s: nc.all_reduce(src.data_ptr(), dst.data_ptr(), src.numel(), 0, 0,
                                                              s))
        wk.wait()
    for v in (3.0, 5.0):
        src.fill_(v)
        g.replay()
        torch.cuda.synchronize()
        assert float(dst.sum()) == v * 4096


def _collectives_rank(rank, world, comm):
    import torch
    dev = comm.device
    x = torch.arange(12, dtype=torch.float32, device=dev) + 100 * rank
    comm.all_reduce(x)
    rs_in = torch.arange(8, dtype=torch.float32, device=dev) * (rank + 1)
    rs_out = torch.empty(8 // world, device=dev)
    comm.reduce_scatter(rs_out, rs_in)
    ag = torch.empty(3 * world, device=dev)
    comm.all_gather(ag, torch.full((3,), float(rank), device=dev))
    bc = torch.full((5,), float(rank + 7), device=dev)
    comm.broadcast(bc, 1)
    a2a_in = torch.arange(4, dtype=torch.float32, device=dev) + 10 * rank
    a2a_out = torch.empty(4, device=dev)
    comm.all_to_all(a2a_out, a2a_in)
    p2p = torch.full((6,), float(rank), device=dev)
    if rank == 0:
        comm.send(p2p, 1)
    else:
        comm.recv(p2p, 0)
    h = comm.all_reduce(torch.ones(3, device=dev), async_op=True)
    h.wait()
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in (x, rs_out, ag, bc, a2a_out, p2p)]


def _rccl_two_ranks(fn, *args):
    try:
        return run_ranks(fn, 2, *args, backend="rccl", timeout=240)
    except RuntimeError as e:
        msg = str(e)
        if "ncclCommInitRank" in msg or "Duplicate" in msg or "duplicate" in msg:
            pytest.skip(f"RCCL does not admit two ranks on one GPU here: {msg[-300:]}")
        raise


def test_rccl_two_ranks_collectives(gpu):
    res = _rccl_two_ranks(_collectives_rank)
    x = np.arange(12, dtype=np.float32)
    for r in (0, 1):
        x_, rs, ag, bc, a2a, p2p = res[r]
        np.testing.assert_array_equal(x_, 2 * x + 100)
        np.testing.assert_array_equal(rs, (np.arange(8) * 3)[r * 4:(r + 1) * 4])
        np.testing.assert_array_equal(ag, [0, 0, 0, 1, 1, 1])
        np.testing.assert_array_equal(bc, np.full(5, 8.0))
        np.testing.assert_array_equal(a2a, [r * 2, r * 2 + 1, 10 + r * 2, 10 + r * 2 + 1])
        np.testing.assert_array_equal(p2p, np.zeros(6))


def _mlp_step(rank, world, comm, steps=3, bf16_grads=False):
    """DistOpt on the GPU: rank r trains on its half of a fixed batch."""
    import torch

    from singa_amd import device, opt, tensor
    from singa_amd.models import mlp
    from singa_amd.parallel import DistOpt

    dev = device.create_rocm_gpu_on(0)
    dev.SetRandSeed(11 + rank)  # different init: attach() must broadcast rank 0's weights
    rng = np.random.RandomState(0)
    X = rng.randn(16, 40).astype(np.float32)
    Y = rng.randint(0, 10, 16).astype(np.int32)
    n = 16 // world
    x = tensor.from_numpy(X[rank * n:(rank + 1) * n], dev)
    y = tensor.from_numpy(Y[rank * n:(rank + 1) * n], dev)
    m = mlp.create_model((64, 48), 10)
    o = opt.SGD(0.1, 0.9)
    if comm is not None:
        o = DistOpt(o, comm=comm, bucket_mb=0.004, first_bucket_mb=0.002,
                    grad_dtype=torch.bfloat16 if bf16_grads else torch.float32)
    m.set_optimizer(o)
    m.compile([x], is_train=True)
    for _ in range(steps):
        m(x, y)
    torch.cuda.synchronize()
    return {k: v.data.float().cpu().numpy() for k, v in m.get_params().items()}


def test_rccl_distopt_equals_single_process_step(gpu):
    """2 ranks x half batch over RCCL == 1 process x full batch (mean loss:
    the averaged bucket all-reduce reproduces the full-batch gradient)."""
    res = _rccl_two_ranks(_mlp_step)
    for k in res[0]:
        np.testing.assert_allclose(res[0][k], res[1][k], rtol=0, atol=0, err_msg=k)  # replicas bit-identical
    ref = _single_process(gpu)
    for k in ref:
        np.testing.assert_allclose(res[0][k], ref[k], rtol=2e-5, atol=2e-6, err_msg=k)


def _single_process(gpu):
    """The full-batch reference step (rank 0's init, world 1, no DistOpt)."""
    import torch

    from singa_amd import device, opt, tensor
    from singa_amd.models import mlp

    dev = device.create_rocm_gpu_on(0)
    dev.SetRandSeed(11)
    rng = np.random.RandomState(0)
    X = rng.randn(16, 40).astype(np.float32)
    Y = rng.randint(0, 10, 16).astype(np.int32)
    m = mlp.create_model((64, 48), 10)
    m.set_optimizer(opt.SGD(0.1, 0.9))
    x, y = tensor.from_numpy(X, dev), tensor.from_numpy(Y, dev)
    m.compile([x], is_train=True)
    for _ in range(3):
        m(x, y)
    torch.cuda.synchronize()
    return {k: v.data.float().cpu().numpy() for k, v in m.get_params().items()}


def test_distopt_gloo_gpu_equals_single_process_step(gpu):
    """The same equivalence with the torch gloo communicator carrying device
    tensors (the fallback path), so it is pinned even where RCCL refuses two
    ranks on one GPU."""
    res = run_ranks(_mlp_step, 2)
    ref = _single_process(gpu)
    for k in ref:
        np.testing.assert_allclose(res[0][k], ref[k], rtol=2e-5, atol=2e-6, err_msg=k)
        np.testing.assert_allclose(res[1][k], ref[k], rtol=2e-5, atol=2e-6, err_msg=k)


def test_rccl_bf16_gradient_buckets(gpu):
    res = _rccl_two_ranks(_mlp_step, 3, True)
    ref = _single_process(gpu)
    for k in ref:
        np.testing.assert_allclose(res[0][k], ref[k], rtol=2e-2, atol=2e-3, err_msg=k)


def test_sparse_topk_threshold_is_exact(gpu):
    from singa_amd.ops import glue as G
    g = torch.randn(1_000_003, generator=torch.Generator().manual_seed(5))
    for k in (1, 17, 5000, 1_000_003):
        thr = G.kth_largest_abs(g.to(gpu), k)
        ref = g.abs().kthvalue(g.numel() - k + 1).values
        assert float(thr) == float(ref)


# ----------------------------------------------- loopback ranks on one GPU
# N ranks as threads of this process, each on its own HIP stream, over the
# native loopback communicator behind the REAL RcclCommunicator: the wrapper's
# comm-stream fork / join, DistOpt's fp32 and bf16 bucket staging and the
# sharded EASGD centre at the world sizes of the 8-GPU run
# (csrc/comm/loop_comm.cpp, parallel/loop.py).
_INIT = __import__("threading").Lock()


def _mlp_step_locked(rank, world, comm, steps, bf16):
    """_mlp_step for rank threads sharing one device object: the seeded
    parameter init of each rank runs under a lock (the device RNG is shared),
    so rank 0's initial weights -- which DistOpt broadcasts -- are exactly the
    single-process reference's."""
    from singa_amd import device, opt, tensor
    from singa_amd.models import mlp
    from singa_amd.parallel import DistOpt

    dev = device.create_rocm_gpu_on(0)
    rng = np.random.RandomState(0)
    X = rng.randn(16, 40).astype(np.float32)
    Y = rng.randint(0, 10, 16).astype(np.int32)
    n = 16 // world
    x = tensor.from_numpy(X[rank * n:(rank + 1) * n], dev)
    y = tensor.from_numpy(Y[rank * n:(rank + 1) * n], dev)
    m = mlp.create_model((64, 48), 10)
    with _INIT:
        dev.SetRandSeed(11 + rank)
        m.compile([x], is_train=False)
        torch.cuda.current_stream().synchronize()
    m.set_optimizer(DistOpt(opt.SGD(0.1, 0.9), comm=comm, bucket_mb=0.004, first_bucket_mb=0.002,
                            grad_dtype=torch.bfloat16 if bf16 else torch.float32))
    m.compile([x], is_train=True)
    for _ in range(steps):
        m(x, y)
    torch.cuda.current_stream().synchronize()
    return {k: v.data.float().cpu().numpy() for k, v in m.get_params().items()}


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("bf16", [False, True])
def test_loopback_distopt_equals_single_process_step(gpu, world, bf16):
    from singa_amd.parallel.loop import run_ranks as loop_ranks

    res = loop_ranks(_mlp_step_locked, world, 3, bf16, device=torch.device("cuda", 0), timeout_s=120.0)
    ref = _single_process(gpu)
    for k in ref:
        for r in range(world):
            np.testing.assert_array_equal(res[r][k], res[0][k], err_msg=f"{k} rank {r}")  # replicas identical
        if bf16:
            np.testing.assert_allclose(res[0][k], ref[k], rtol=2e-2, atol=2e-3, err_msg=k)
        else:
            np.testing.assert_allclose(res[0][k], ref[k], rtol=2e-5, atol=2e-6, err_msg=k)


def _easgd_gpu_rank(rank, world, comm, sharded):
    from singa_amd.opt import SGD
    from singa_amd.parallel.easgd import ElasticSync
    from singa_amd.tensor import Tensor

    from singa_amd import device
    dev = device.create_rocm_gpu_on(0)
    g = torch.Generator().manual_seed(0)
    p = Tensor(device=dev, data=torch.randn(1000, generator=g).to(gpu_dev()), requires_grad=True, stores_grad=True)
    q = Tensor(device=dev, data=torch.randn(30, 7, generator=g).to(gpu_dev()), requires_grad=True, stores_grad=True)
    st = SGD(0.1).attach([p, q])
    es = ElasticSync(st, comm, moving_rate=0.5, sharded=sharded)
    es.bootstrap()
    c0 = st.w.clone()
    st.w.add_(float(rank + 1))
    wb = st.w.clone()
    es.sync()
    full = torch.empty_like(st.w)
    if es.sharded:
        comm.all_gather(full, es.centre)
    else:
        full.copy_(es.centre)
    torch.cuda.current_stream().synchronize()
    return c0.cpu().numpy(), wb.cpu().numpy(), st.w.cpu().numpy(), full.cpu().numpy(), es.alpha


def gpu_dev():
    return torch.device("cuda", 0)


@pytest.mark.parametrize("sharded", [False, True])
def test_loopback_easgd_eight_ranks(gpu, sharded):
    """Sharded (reduce-scatter / all-gather over 8 ranks) and replicated
    centres follow c' = c + sum_r alpha (w_r - c), w_r' = w_r - alpha (w_r - c)."""
    from singa_amd.parallel.loop import run_ranks as loop_ranks

    res = loop_ranks(_easgd_gpu_rank, 8, sharded, device=gpu_dev(), timeout_s=120.0)
    c0, alpha = res[0][0], res[0][4]
    ds = [alpha * (wb - c0) for _, wb, _, _, _ in res]
    for r, (_, wb, wa, c, _) in enumerate(res):
        np.testing.assert_allclose(wa, wb - ds[r], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(c, c0 + sum(ds), rtol=1e-5, atol=1e-5)


def _easgd_rounds_rank(rank, world, comm, sharded, overlap):
    from singa_amd.opt import SGD
    from singa_amd.parallel.easgd import ElasticSync
    from singa_amd.tensor import Tensor

    from singa_amd import device
    dev = device.create_rocm_gpu_on(0)
    g = torch.Generator().manual_seed(0)
    p = Tensor(device=dev, data=torch.randn(4096, generator=g).to(gpu_dev()), requires_grad=True, stores_grad=True)
    st = SGD(0.1).attach([p])
    es = ElasticSync(st, comm, moving_rate=0.9, sharded=sharded, overlap=overlap)
    es.bootstrap()
    drift = torch.randn(4096, generator=torch.Generator().manual_seed(rank + 1)).to(gpu_dev())
    for step in range(6):
        st.w.add_(drift)  # "training" between syncs, on the compute stream
        es.sync()
    es.wait()
    full = torch.empty_like(st.w)
    if es.sharded:
        comm.all_gather(full, es.centre)
    else:
        full.copy_(es.centre)
    torch.cuda.current_stream().synchronize()
    return st.w.cpu().numpy(), full.cpu().numpy(), es._pending is None


@pytest.mark.parametrize("sharded", [False, True])
def test_loopback_easgd_overlapped_equals_synchronous(gpu, sharded):
    """The overlapped exchange (comm stream, joined at the next sync) gives
    the synchronous schedule's weights and centre exactly, at 4 ranks."""
    from singa_amd.parallel.loop import run_ranks as loop_ranks

    sync = loop_ranks(_easgd_rounds_rank, 4, sharded, False, device=gpu_dev(), timeout_s=120.0)
    ovl = loop_ranks(_easgd_rounds_rank, 4, sharded, True, device=gpu_dev(), timeout_s=120.0)
    for r in range(4):
        np.testing.assert_array_equal(ovl[r][0], sync[r][0])
        np.testing.assert_array_equal(ovl[r][1], sync[r][1])
        assert ovl[r][2]


def _easgd_pp_rank(rank, world, comm, per_param):
    from singa_amd import device
    from singa_amd.opt import SGD
    from singa_amd.parallel.easgd import ElasticSync
    from singa_amd.tensor import Tensor

    dev = device.create_rocm_gpu_on(0)
    g = torch.Generator().manual_seed(0)
    ps = [Tensor(device=dev, data=torch.randn(n, generator=g).to(gpu_dev()), requires_grad=True, stores_grad=True)
          for n in (3000, 517, 4096, 64, 2000)]
    o = SGD(0.05, 0.9, weight_decay=1e-4)
    st = o.attach(ps)
    es = ElasticSync(st, comm, moving_rate=0.9, sync_frequency=2, overlap=True, bucket_mb=0.005)
    es.bootstrap()
    gg = torch.Generator().manual_seed(rank + 1)
    for step in range(7):
        grads = torch.randn(st.numel, generator=gg).to(gpu_dev())
        if per_param:
            es.wait_params(st.params)  # (the forward's per-layer joins)
            es.begin_step(o, step)
            st.g.copy_(grads)
            for p in st.params:  # the backward: store order = completion order
                es.on_grad(p)
            es.end_step()
        else:
            st.g.copy_(grads)
            o.update()
            o.step()
            if es.sync_now(step + 1):
                es.sync()
    es.wait()
    torch.cuda.current_stream().synchronize()
    nb = len(es._buckets) if es._buckets else 0
    return st.w.cpu().numpy(), es.centre.cpu().numpy(), es.nsync, nb


def test_loopback_easgd_per_param_equals_whole_buffer(gpu):
    """Per-bucket update + elastic exchange forked onto the comm stream as the
    'backward' completes each bucket (events joined per parameter) == the
    whole-buffer update + sync, exactly, at 4 ranks."""
    from singa_amd.parallel.loop import run_ranks as loop_ranks

    pp = loop_ranks(_easgd_pp_rank, 4, True, device=gpu_dev(), timeout_s=120.0)
    wb = loop_ranks(_easgd_pp_rank, 4, False, device=gpu_dev(), timeout_s=120.0)
    for r in range(4):
        assert pp[r][3] >= 3 and pp[r][2] == wb[r][2] >= 3
        np.testing.assert_array_equal(pp[r][0], wb[r][0])
        np.testing.assert_array_equal(pp[r][1], wb[r][1])
