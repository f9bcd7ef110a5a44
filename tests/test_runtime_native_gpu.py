"""Framework-owned execution substrate on the MI355X: every activation and
temporary of a training step comes from the native HBM pool (no PyTorch
allocation inside a step), the pool's stream-ordered reuse and
record_stream, native streams / events, and the native HIP-graph step
executor (csrc/mem/pool.cpp, csrc/mem/stream_graph.cpp, singa_amd/memory.py,
singa_amd/stream.py).  Reference counterparts: mshadow AllocSpace / FreeSpace
(include/mshadow/tensor.h:206-385) and SyncedMemory (src/utils/blob.cc:83-298)."""
import gc

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_allocs():
    return torch.cuda.memory_stats().get("allocation.all.allocated", 0)


def _resnet_step_setup(gpu, depth=18, B=4, graph=False):
    from singa_amd import device, opt, tensor
    from singa_amd.models import resnet

    dev = device.create_rocm_gpu_on(0)
    dev.SetRandSeed(0)
    m = resnet.create_model(depth, num_classes=10, compute_dtype=torch.bfloat16)
    m.set_optimizer(opt.SGD(0.01, 0.9))
    rng = np.random.RandomState(0)
    x = tensor.from_numpy(rng.standard_normal((B, 3, 64, 64)).astype(np.float32), dev)
    y = tensor.from_numpy(rng.randint(0, 10, B).astype(np.int32), dev)
    m.compile([x], is_train=True, use_graph=graph)
    return m, x, y


def test_training_step_allocates_nothing_through_pytorch(gpu):
    """After warm-up, a ResNet-18 training step makes zero PyTorch allocator
    allocations: activations, temporaries and workspaces are native pool
    blocks, and the pool's peak accounts for them."""
    from singa_amd import memory

    m, x, y = _resnet_step_setup(gpu)
    for _ in range(2):
        m(x, y)
    torch.cuda.synchronize()
    memory.reset_peak(gpu)
    base_in_use = memory.stats(gpu)["in_use_bytes"]
    a0 = _torch_allocs()
    s0 = memory.stats(gpu)["allocs"]
    m(x, y)
    torch.cuda.synchronize()
    st = memory.stats(gpu)
    assert _torch_allocs() == a0, "a PyTorch allocation inside the training step"
    assert st["allocs"] - s0 > 100  # the step's activations / temporaries came from the native pool
    assert st["peak_in_use_bytes"] > base_in_use  # ... and the pool's peak accounts for them


def test_native_stream_event_roundtrip(gpu):
    from singa_amd import stream
    from singa_amd.ops import glue as G

    s = stream.Stream(gpu, priority=-1)
    x = torch.zeros(1 << 22, device=gpu)
    e0, e1 = stream.Event(timing=True), stream.Event(timing=True)
    s.wait_stream(torch.cuda.current_stream())
    with s:
        assert torch.cuda.current_stream().cuda_stream == s.handle
        e0.record()
        for _ in range(10):
            G.binary("add", x, 1.0, out=x)
        e1.record()
    e1.wait()  # current stream joins s
    assert float(x[0]) == 10.0 and float(x[-1]) == 10.0
    e1.synchronize()
    assert e1.query() and e0.elapsed_time(e1) >= 0.0
    s.synchronize()


def test_record_stream_defers_reuse_until_other_stream_done(gpu):
    from singa_amd import memory, stream
    from singa_amd.ops import glue as G

    s = stream.Stream(gpu)
    t = memory.empty((16 << 20,), dtype=torch.float32, device=gpu)
    p = t.data_ptr()
    s.wait_stream(torch.cuda.current_stream())
    with s:
        for _ in range(30):
            G.fill_(t, 2.0)  # queued on s
    memory.record_stream(t, s)
    del t
    gc.collect()
    u = memory.empty((16 << 20,), dtype=torch.float32, device=gpu)
    if u.data_ptr() == p:  # only once s finished its fills
        assert s.query()
    s.synchronize()
    del u


def test_native_step_graph_equals_eager(gpu):
    """Model(use_graph=True) captures the step with the native StepGraph
    (hipStreamBeginCapture on a framework stream, private native pool);
    replaying it trains exactly like eager execution.  Deterministic kernel
    mode: with the atomic split-K / statistics sums the two runs drift apart
    within a few steps of this tiny-batch (B=4) fit (measured: 1 in 3 runs
    past 2e-3 on the second step's loss)."""
    from singa_amd import stream
    from singa_amd.ops import native as NN

    res = []
    NN.lib().set_deterministic(1)
    try:
        for graph in (False, True):
            m, x, y = _resnet_step_setup(gpu, graph=graph)
            losses = [float(m(x, y)[1].data.float()) for _ in range(5)]
            torch.cuda.synchronize()
            if graph:
                g = m._graphs["train"][0]
                assert isinstance(g, stream.StepGraph) and g.nodes > 100
            res.append((losses, {k: v.data.float().cpu() for k, v in m.get_params().items()}))
            if graph:
                m.reset_graph()
    finally:
        NN.lib().set_deterministic(0)
    (l0, p0), (l1, p1) = res
    np.testing.assert_allclose(l1, l0, rtol=2e-3, atol=2e-3)
    for k in p0:
        torch.testing.assert_close(p1[k], p0[k], rtol=2e-2, atol=2e-3)


def test_graph_private_pool_released(gpu):
    from singa_amd import memory

    m, x, y = _resnet_step_setup(gpu, graph=True)
    for _ in range(4):
        m(x, y)
    torch.cuda.synchronize()
    r0 = memory.stats(gpu)["reserved_bytes"]
    m.reset_graph()
    gc.collect()
    torch.cuda.synchronize()
    assert memory.stats(gpu)["reserved_bytes"] < r0  # the graph's private blocks went back to the driver
