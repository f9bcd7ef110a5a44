"""singa_amd.data iterators and singa_amd.metric (CPU)."""
import os

import numpy as np
import pytest

from test_tools_cpu import _write_idx


def test_shard_iterator(tmp_path):
    from singa_amd import data, loader

    ip, lp, imgs, labs = _write_idx(str(tmp_path), n=40)
    folder = str(tmp_path / "s")
    loader.load_mnist(ip, lp, folder)
    it = data.ShardIterator(folder, 8, scale=1 / 255.0)
    assert len(it) == 5
    x, y = next(it)
    assert x.shape == (8, 6, 6) and y.dtype == np.int32
    np.testing.assert_allclose(x, imgs[:8] / 255.0, rtol=1e-6)
    np.testing.assert_array_equal(y, labs[:8])
    with pytest.raises(FileNotFoundError):
        data.ShardIterator(str(tmp_path / "none"), 8)


def test_array_iterator_and_synthetic():
    from singa_amd import data

    x = np.arange(20, dtype=np.float32).reshape(10, 2)
    y = np.arange(10, dtype=np.int32)
    seen = []
    for bx, by in data.ArrayIterator(x, y, 3, shuffle=True, seed=1):
        np.testing.assert_array_equal(bx[:, 0] / 2, by)
        seen += list(by)
    assert len(seen) == 9 and len(set(seen)) == 9
    assert len(list(data.ArrayIterator(x, y, 3, drop_last=False))) == 4
    s = data.SyntheticImages(4, (3, 8, 8), 10)
    a, la = next(s)
    assert a.shape == (4, 3, 8, 8) and la.max() < 10
    assert next(s)[0] is a  # fixed batch reused


def test_image_batch_iter(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    from singa_amd import data
    import random

    lst = []
    for i in range(6):
        p = tmp_path / f"{i}.png"
        PIL.fromarray(np.full((10, 12, 3), i * 20, np.uint8)).save(p)
        lst.append(f"{p.name} {i}")
    (tmp_path / "list.txt").write_text("\n".join(lst))
    rng = random.Random(0)
    it = data.ImageBatchIter(str(tmp_path / "list.txt"), 3, image_folder=str(tmp_path),
                             transform=lambda a: data.crop_mirror(a, 8, True, rng).astype(np.float32))
    it.start()
    x, y = next(it)
    it.end()
    assert x.shape == (3, 3, 8, 8)
    for img, lab in zip(x, y):
        assert np.all(img == lab * 20)


def test_metrics():
    from singa_amd import metric

    x = np.array([[0.1, 0.7, 0.2], [0.5, 0.3, 0.2], [0.2, 0.3, 0.5], [0.3, 0.4, 0.3]], np.float32)
    y = np.array([1, 1, 2, 0])
    assert metric.Accuracy().evaluate(x, y) == pytest.approx(0.5)
    assert metric.Accuracy(top_k=2).evaluate(x, y) == pytest.approx(1.0)
    # predictions 1,0,2,1 -> precision class0: 0/1, class1: 1/2, class2: 1/1
    assert metric.Precision().evaluate(x, y) == pytest.approx((0 + 0.5 + 1) / 3)
    assert metric.Recall().evaluate(x, y) == pytest.approx((0 + 0.5 + 1) / 3)
    import torch
    assert metric.Accuracy().evaluate(torch.from_numpy(x), torch.from_numpy(y)) == pytest.approx(0.5)
    from singa_amd import module, model
    assert module.Module is model.Model


def test_native_lmdb_reader_and_datum_layer(tmp_path):
    """kLMDBData without liblmdb: the native reader walks a multi-level
    B+tree (branch + leaf pages, an overflow value), picks the newer meta
    page, decodes Caffe Datums, and the data source wraps at the end."""
    from lmdb_writer import datum, write_lmdb

    from singa_amd import _core
    from singa_amd.runtime.layers import DataSource

    rng = np.random.RandomState(0)
    items = []
    for i in range(300):
        px = rng.randint(0, 256, size=3 * 8 * 8).astype(np.uint8).tobytes()
        items.append((b"%08d" % i, datum(3, 8, 8, px, i % 7)))
    big = (b"zz_big", datum(3, 40, 40, rng.randint(0, 256, size=3 * 40 * 40).astype(np.uint8).tobytes(), 3))
    write_lmdb(str(tmp_path / "db"), items + [big], leaf_limit=16)
    r = _core.LmdbReader(str(tmp_path / "db"))
    assert r.count() == 301
    got = []
    while True:
        kv = r.next()
        if kv is None:
            break
        got.append(kv)
    assert [k for k, _ in got] == sorted(k for k, _ in items + [big])
    assert dict(got)[b"00000042"] == dict(items)[b"00000042"] and dict(got)[b"zz_big"] == big[1]
    d = _core.decode_datum(dict(items)[b"00000042"])
    assert d["shape"] == [3, 8, 8] and d["label"] == 42 % 7 and not d["encoded"]
    # data source over the 300 uniform records (wraps around after the last)
    write_lmdb(str(tmp_path / "db2"), items, leaf_limit=16)
    src = DataSource(str(tmp_path / "db2"), batch=128)
    assert src.kind == "lmdb" and src.shape == (3, 8, 8)
    labs = np.concatenate([src.next()[1] for _ in range(3)])
    assert np.array_equal(labs, np.array([i % 7 for i in range(300)] + [i % 7 for i in range(84)]))
    img, _ = DataSource(str(tmp_path / "db2"), batch=2).next()
    px1 = np.frombuffer(_core.decode_datum(items[1][1])["pixel"], np.uint8).astype(np.float32)
    assert np.array_equal(img[1].ravel(), px1)
