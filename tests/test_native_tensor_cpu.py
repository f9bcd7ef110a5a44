"""The framework-owned tensor handle (_C.mem.Tensor, csrc/mem/pool.cpp):
pool storage + byte offset + shape / strides / dtype / device, native views,
DLPack export and import -- checked against PyTorch views of the same bytes
(host pool here; tests/test_native_tensor_gpu.py runs the device pool)."""
import numpy as np
import pytest
import torch

from singa_amd import memory as mem
from singa_amd.ops import native as N

pytestmark = pytest.mark.skipif(not N.available() or not hasattr(N.lib().mem, "Tensor"),
                                reason="needs the _C extension")


def _filled(shape, dtype=torch.float32):
    h = mem.empty_native(shape, dtype)
    t = mem.to_torch(h)
    t.copy_(torch.arange(t.numel(), dtype=torch.float32).reshape(shape).to(dtype))
    return h, t


def test_empty_metadata_and_layouts():
    h = mem.empty_native((2, 3, 4, 5), torch.bfloat16)
    assert h.shape == (2, 3, 4, 5) and h.strides == (60, 20, 5, 1) and h.ndim == 4
    assert h.dtype == (4, 16) and h.itemsize == 2 and h.numel() == 120 and h.nbytes() == 240
    assert h.is_contiguous() and not h.is_channels_last() and h.storage_kind == 1
    c = mem.empty_native((2, 3, 4, 5), torch.float32, channels_last=True)
    assert c.strides == (60, 1, 15, 3) and c.is_channels_last() and not c.is_contiguous()
    assert mem.to_torch(c).is_contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("seed", range(6))
def test_views_match_torch(seed):
    rng = np.random.RandomState(seed)
    h, t = _filled((4, 5, 6))
    for _ in range(6):
        op = rng.randint(7)
        r = t.dim()
        if op == 0 and r > 1:
            dims = list(rng.permutation(r))
            h, t = h.permute(dims), t.permute(*dims)
        elif op == 1:
            d = rng.randint(r)
            n = t.shape[d]
            a, b, s = rng.randint(0, n), n, rng.randint(1, 3)
            h, t = h.slice(d, a, b, s), t[(slice(None),) * d + (slice(a, b, s),)]
        elif op == 2 and r > 1 and min(t.shape) > 0:
            d = rng.randint(r)
            i = rng.randint(t.shape[d])
            h, t = h.select(d, i), t.select(d, i)
        elif op == 3:
            d = rng.randint(r + 1)
            h, t = h.unsqueeze(d), t.unsqueeze(d)
        elif op == 4 and 1 in t.shape:
            d = list(t.shape).index(1)
            h, t = h.squeeze(d), t.squeeze(d)
        elif op == 5 and r > 1:
            a, b = rng.randint(r), rng.randint(r)
            h, t = h.transpose(a, b), t.transpose(a, b)
        elif op == 6 and t.is_contiguous():
            h, t = h.reshape([-1]), t.reshape(-1)
        assert h.shape == tuple(t.shape) and h.strides == tuple(t.stride()), (op, h.shape, t.shape)
        assert h.data_ptr() == t.data_ptr() or t.numel() == 0
        if t.numel():
            assert torch.equal(mem.to_torch(h), t)


def test_expand_and_as_strided():
    h, t = _filled((3, 1))
    e = h.expand([2, 3, 4])
    assert e.strides == (0, 1, 0) and torch.equal(mem.to_torch(e), t.expand(2, 3, 4))
    a = h.as_strided([2, 2], [1, 1], 0)
    assert torch.equal(mem.to_torch(a), torch.as_strided(t, (2, 2), (1, 1), 0))
    with pytest.raises(IndexError):
        h.as_strided([3, 3], [1, 1], 0)  # reaches element 4 of a 3-element storage


def test_storage_outlives_views_and_imports():
    h, t = _filled((8, 8))
    v = h.slice(0, 2, 4)
    refs = h.storage_refs
    del h
    assert v.storage_refs == refs - 1
    tv = mem.to_torch(v)
    del v, t
    assert torch.equal(tv, torch.arange(16, 32, dtype=torch.float32).reshape(2, 8))
    x = torch.randn(5, 7)
    n = mem.native(x)  # zero-copy import of a foreign (PyTorch-allocated) buffer
    assert n.storage_kind == 3 and n.data_ptr() == x.data_ptr() and n.shape == (5, 7)
    assert np.array_equal(np.from_dlpack(n.transpose(0, 1)), x.numpy().T)


def test_errors():
    h, _ = _filled((4, 6))
    with pytest.raises(ValueError):
        h.slice(1, 0, 6, 2).reshape([12])  # not contiguous: needs a copy
    with pytest.raises(ValueError):
        h.reshape([5, -1])
    with pytest.raises(IndexError):
        h.select(0, 4)
    with pytest.raises(ValueError):
        h.permute([0, 0])


def test_singa_tensor_round_trip():
    from singa_amd import tensor

    x = tensor.from_numpy(np.arange(12, dtype=np.float32).reshape(3, 4))
    h = x.native
    assert h.shape == (3, 4) and h.data_ptr() == x.data.data_ptr()
    y = tensor.Tensor.from_native(h.transpose(0, 1))
    assert y.shape == (4, 3) and np.array_equal(tensor.to_numpy(y), np.arange(12).reshape(3, 4).T)
