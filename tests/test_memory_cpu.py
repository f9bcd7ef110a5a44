"""Native memory pools (csrc/mem/pool.cpp, singa_amd/memory.py): host pool
blocks handed to PyTorch as DLPack tensors, reuse through the size-class
cache, the parameter store living in them, and parity with PyTorch's
allocator (reference: mshadow AllocSpace/FreeSpace, include/mshadow/tensor.h:206-385;
Blob/SyncedMemory, src/utils/blob.cc:83-298)."""
import gc

import numpy as np
import pytest
import torch

from singa_amd import memory

pytestmark = pytest.mark.skipif(not memory.enabled(), reason="_C not built")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.int32, torch.int64,
                                   torch.uint8, torch.float64])
def test_host_blocks_are_framework_owned_tensors(dtype):
    t = memory.empty((3, 5, 7), dtype)
    assert t.shape == (3, 5, 7) and t.dtype == dtype and t.is_contiguous() and not t.is_cuda
    assert t.data_ptr() % 64 == 0
    t.fill_(3)
    assert float(t.float().sum()) == 3 * 105


def test_host_pool_reuses_freed_blocks():
    before = memory.stats()
    a = memory.empty((1000,), torch.float32)
    pa = a.data_ptr()
    del a
    gc.collect()
    b = memory.empty((999,), torch.float32)  # same 512-byte size class
    after = memory.stats()
    assert b.data_ptr() == pa
    assert after["cache_hits"] >= before["cache_hits"] + 1
    assert after["frees"] >= before["frees"] + 1
    v = b[10:20].view(2, 5)  # views keep the block alive
    del b
    gc.collect()
    assert memory.stats()["in_use_bytes"] >= 4096
    del v
    gc.collect()


def test_zeros_and_views():
    z = memory.zeros((4, 6), torch.float32)
    assert float(z.abs().sum()) == 0.0
    z[1:3, 2:4] = 1.0
    assert float(z.sum()) == 4.0


def _train(native):
    import os

    from singa_amd import device, opt, tensor
    from singa_amd.models import mlp
    os.environ["SINGA_AMD_NATIVE_MEM"] = "1" if native else "0"
    try:
        dev = device.get_default_device()
        dev.SetRandSeed(0)
        rng = np.random.RandomState(0)
        x = tensor.from_numpy(rng.rand(32, 784).astype(np.float32))
        y = tensor.from_numpy(rng.randint(0, 10, 32).astype(np.int32))
        m = mlp.create_model((64,), 10)
        m.set_optimizer(opt.Adam(0.01))
        m.compile([x], is_train=True)
        m.train()
        for _ in range(3):
            m(x, y)
        st = m.optimizer.store
        return {k: v.data.clone() for k, v in m.get_params().items()}, st
    finally:
        os.environ.pop("SINGA_AMD_NATIVE_MEM", None)


def test_param_store_in_native_pool_trains_identically():
    before = memory.stats()["allocs"]
    p_nat, st = _train(True)
    assert memory.stats()["allocs"] >= before + 4  # w, g, s1, s2
    p_ref, _ = _train(False)
    for k in p_ref:
        assert torch.equal(p_nat[k], p_ref[k]), k
