"""Native HBM pool on the MI355X (csrc/mem/pool.cpp): device blocks as DLPack
tensors, stream-ordered reuse (a block freed with work still queued on its
stream is reused only after that work completed), blocks freed during a
HIP-graph capture never reused, and a training step whose parameter store
lives in the pool equal to one on PyTorch's allocator."""
import gc
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_device_blocks_and_reuse(gpu):
    from singa_amd import memory
    t = memory.empty((1 << 20,), torch.float32, gpu)
    assert t.is_cuda and t.device.index == 0 and t.data_ptr() % 256 == 0
    t.fill_(1.5)
    assert float(t.sum()) == 1.5 * (1 << 20)
    p = t.data_ptr()
    torch.cuda.synchronize()
    del t
    gc.collect()
    torch.cuda.synchronize()
    u = memory.empty((1 << 20,), torch.float32, gpu)
    assert u.data_ptr() == p  # the cached block, after its event completed
    st = memory.stats(gpu)
    assert st["cache_hits"] >= 1 and st["in_use_bytes"] >= 4 << 20
    del u
    gc.collect()


def test_stream_ordered_reuse_waits_for_queued_work(gpu):
    """A block freed while a long kernel still writes it must not be handed
    out again until that kernel finished."""
    from singa_amd import memory
    from singa_amd.ops import glue as G
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        big = memory.empty((64 << 20,), torch.float32, gpu)
        for _ in range(20):
            G.fill_(big, 3.0)  # queued work on s
        p = big.data_ptr()
        del big
        gc.collect()
        st = memory.stats(gpu)
        other = memory.empty((64 << 20,), torch.float32, gpu)
        if other.data_ptr() == p:  # only legal if the queued fills were already done
            assert st["pending_frees"] == 0
    torch.cuda.synchronize()
    del other
    gc.collect()


def test_free_during_capture_is_never_reused(gpu):
    from singa_amd import memory
    from singa_amd.ops import glue as G
    keep = memory.empty((1024,), torch.float32, gpu)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        tmp = memory.empty((4096,), torch.float32, gpu)  # allocated before capture
    torch.cuda.synchronize()
    p = tmp.data_ptr()
    with torch.cuda.graph(g, stream=s):
        G.fill_(keep, 2.0)
        del tmp
        gc.collect()
    g.replay()
    torch.cuda.synchronize()
    again = memory.empty((4096,), torch.float32, gpu)
    assert again.data_ptr() != p
    assert float(keep.sum()) == 2048.0


def _step(native):
    from singa_amd import device, opt, tensor
    from singa_amd.models import mlp
    os.environ["SINGA_AMD_NATIVE_MEM"] = "1" if native else "0"
    try:
        dev = device.create_rocm_gpu_on(0)
        dev.SetRandSeed(3)
        rng = np.random.RandomState(0)
        x = tensor.from_numpy(rng.rand(64, 96).astype(np.float32), dev)
        y = tensor.from_numpy(rng.randint(0, 10, 64).astype(np.int32), dev)
        m = mlp.create_model((128,), 10)
        m.set_optimizer(opt.SGD(0.05, 0.9))
        m.compile([x], is_train=True, use_graph=True)
        m.train()
        for _ in range(4):
            m(x, y)
        torch.cuda.synchronize()
        return {k: v.data.float().cpu() for k, v in m.get_params().items()}
    finally:
        os.environ.pop("SINGA_AMD_NATIVE_MEM", None)


def test_graph_step_with_param_store_in_native_pool(gpu):
    from singa_amd import memory
    a0 = memory.stats(gpu)["allocs"]
    nat = _step(True)
    assert memory.stats(gpu)["allocs"] >= a0 + 3
    ref = _step(False)
    for k in ref:
        assert torch.equal(nat[k], ref[k]), k


def test_synced_blob_head_states(gpu):
    """The reference SyncedMemory state machine on native buffers: lazy
    sides, sync on read, mutable_* makes one side authoritative, and a
    mirror of an external device region (a parameter's store slice)."""
    from singa_amd.memory import SyncedBlob as B
    b = B((4, 5), torch.float32, gpu)
    assert b.head == B.UNINITIALIZED
    h = b.mutable_cpu_data()
    assert b.head == B.HEAD_AT_CPU and float(h.abs().sum()) == 0.0
    h.copy_(torch.arange(20, dtype=torch.float32).reshape(4, 5))
    d = b.gpu_data()
    assert b.head == B.SYNCED and d.is_cuda
    torch.testing.assert_close(d.cpu(), h)
    d2 = b.mutable_gpu_data()
    d2.mul_(2.0)
    assert b.head == B.HEAD_AT_GPU
    torch.testing.assert_close(b.cpu_data(), h * 0 + torch.arange(20.).reshape(4, 5) * 2)
    assert b.head == B.SYNCED
    # mirror of an existing device slice: host edits land in the slice
    flat = torch.arange(30, dtype=torch.float32, device=gpu)
    m = B(None, like=flat[10:20])
    assert m.head == B.HEAD_AT_GPU
    hv = m.mutable_cpu_data()
    torch.testing.assert_close(hv, torch.arange(10, 20, dtype=torch.float32))
    hv.fill_(-1.0)
    m.gpu_data()
    torch.cuda.synchronize()
    assert float(flat[10:20].sum()) == -10.0 and float(flat[:10].sum()) == 45.0


def test_ps_sync_on_gpu_stores_through_synced_blobs(gpu):
    """EASGD through the native PS with device parameter stores: each
    parameter's host mirror is a SyncedBlob over its store slice."""
    from singa_amd import device, opt
    from singa_amd.parallel.ps import ParamServer, PSClient, PSSync
    from singa_amd.tensor import Tensor

    dev = device.create_rocm_gpu_on(0)
    s = ParamServer(0, 2)
    try:
        ep = [f"127.0.0.1:{s.port}"]

        def store_for(v):
            ps = [Tensor(device=dev, data=torch.full((4, 3), v, device=gpu)),
                  Tensor(device=dev, data=torch.full((7,), v, device=gpu))]
            for p in ps:
                p.requires_grad = p.stores_grad = True
            return opt.SGD(0.1).attach(ps)

        st0, st1 = store_for(1.0), store_for(5.0)
        sy0 = PSSync(st0, PSClient(ep), 0, 2, moving_rate=0.5)
        sy1 = PSSync(st1, PSClient(ep), 1, 2, moving_rate=0.5)
        assert all(b is not None for b in sy1._blobs)
        sy0.bootstrap()
        sy1.bootstrap()
        torch.cuda.synchronize()
        assert all(bool(torch.all(p.data == 1.0)) for p in st1.params)
        for p in st1.params:
            p.data.fill_(3.0)
        sy1.sync()
        torch.cuda.synchronize()
        assert all(torch.allclose(p.data, torch.full_like(p.data, 2.5)) for p in st1.params)
        assert np.allclose(s.value(0), 1.5) and np.allclose(s.value(1), 1.5)
        # group 0 trains after its bootstrap Put: the exchange must see the
        # trained device weights, not the host copy taken at bootstrap
        for p in st0.params:
            p.data.fill_(7.0)
        sy0.sync()
        torch.cuda.synchronize()
        assert all(torch.allclose(p.data, torch.full_like(p.data, 5.625)) for p in st0.params)
        assert np.allclose(s.value(0), 2.875) and np.allclose(s.value(1), 2.875)
        sy0.client.stop()
        sy1.client.stop()
        assert s.wait_stop(5.0)
    finally:
        s.close()
