"""The framework-owned tensor handle on the device pool: HBM storage
(stream-ordered), native views of a tensor a kernel wrote, DLPack export to
the kernel wrappers and back, and the storage returning to the pool when the
last view dies."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_device_handle_views_and_lifetime(gpu):
    from singa_amd import memory as mem
    from singa_amd.ops import glue as G

    dev = torch.device(gpu)
    before = mem.stats(dev)["in_use_bytes"]
    h = mem.empty_native((64, 32, 8, 8), torch.bfloat16, device=dev, channels_last=True)
    assert h.storage_kind == 0 and h.device[1] == (dev.index or 0) and h.is_channels_last()
    assert mem.stats(dev)["in_use_bytes"] >= before + 64 * 32 * 8 * 8 * 2
    t = mem.to_torch(h)
    assert t.is_cuda and t.data_ptr() == h.data_ptr() and t.is_contiguous(memory_format=torch.channels_last)
    G.copy_(t, torch.randn(64, 32, 8, 8, device=dev).bfloat16())  # a native copy kernel writes through the view
    v = h.slice(0, 3, 40, 2).select(1, 5).transpose(1, 2)
    tv = t[3:40:2].select(1, 5).transpose(1, 2)
    assert v.shape == tuple(tv.shape) and v.strides == tuple(tv.stride()) and v.data_ptr() == tv.data_ptr()
    assert torch.equal(mem.to_torch(v), tv)
    s = G.reduce(mem.to_torch(h.reshape([-1]) if h.is_contiguous() else h.permute([0, 2, 3, 1]).reshape([-1])),
                 None, "sum")
    torch.testing.assert_close(s.float(), t.float().sum(), rtol=2e-2, atol=1.0)
    torch.cuda.synchronize()
    del t, tv, v, h
    torch.cuda.synchronize()
    assert mem.stats(dev)["in_use_bytes"] <= before + 4096  # the block went back to the pool
