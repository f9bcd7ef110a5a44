"""Data pipeline (SINGA ``singa.data`` + the reference's data layers C21/C28):

* :class:`ShardIterator` -- batches from a Shard folder written by
  :mod:`singa_amd.loader` (bit-compatible with the reference ``shard.dat``),
  decoded by the native prefetch thread (``_core.Prefetcher``) while the GPU
  computes;
* :class:`ArrayIterator` -- shuffled mini-batches over in-memory arrays;
* :class:`ImageBatchIter` -- SINGA-style folder/list image iterator with a
  transform callback (PIL decode, crop / mirror augmentation, normalisation:
  the reference RGBImageLayer's crop+mirror+scale, F15);
* :class:`SyntheticImages` -- ImageNet / MNIST-shaped random batches (the
  benchmarks use it: there is no dataset download in this environment);
* :class:`DevicePrefetcher` -- overlaps host->device copies with compute on a
  side HIP stream (pinned staging, double buffered).
"""
from __future__ import annotations

import os
import queue
import random
import threading
from typing import Callable, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import memory as _mem
from . import stream as _stream


class ArrayIterator:
    def __init__(self, x: np.ndarray, y: np.ndarray, batch_size: int, shuffle: bool = True, drop_last: bool = True,
                 seed: int = 0):
        assert len(x) == len(y)
        self.x, self.y, self.bs = x, y, batch_size
        self.shuffle, self.drop_last = shuffle, drop_last
        self.rng = np.random.RandomState(seed)

    def __len__(self):
        n = len(self.x)
        return n // self.bs if self.drop_last else (n + self.bs - 1) // self.bs

    def __iter__(self) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
        idx = self.rng.permutation(len(self.x)) if self.shuffle else np.arange(len(self.x))
        for b in range(len(self)):
            j = idx[b * self.bs:(b + 1) * self.bs]
            yield self.x[j], self.y[j]


class ShardIterator:
    """Mini-batches (float32 images [B, *shape], int32 labels [B]) from a
    Shard; pixels are decoded UNSIGNED and scaled: x = pixel*scale + bias."""

    def __init__(self, folder: str, batch_size: int, scale: float = 1.0, bias: float = 0.0, loop: bool = True):
        from . import _core

        if not os.path.exists(os.path.join(folder, "shard.dat")):
            raise FileNotFoundError(f"no shard.dat in {folder}")
        sh = _core.Shard(folder, _core.kRead)
        first = sh.next()
        if first is None:
            raise ValueError(f"empty shard {folder}")
        rec = _core.decode_record(first[1])
        self.shape = tuple(rec["shape"]) if rec["shape"] else (len(rec["data"]) or len(rec["pixel"]),)
        self.dim = int(np.prod(self.shape))
        self.count = sh.count()
        self.bs = batch_size
        self.pf = _core.Prefetcher(folder, batch_size, self.dim, scale, bias, loop)

    def __len__(self):
        return self.count // self.bs

    def __iter__(self):
        return self

    def __next__(self) -> Tuple[np.ndarray, np.ndarray]:
        img = np.empty((self.bs, self.dim), np.float32)
        lab = np.empty((self.bs,), np.int32)
        n = self.pf.next(img, lab)
        if n == 0:
            raise StopIteration
        return img[:n].reshape((n,) + self.shape), lab[:n]


def crop_mirror(img: np.ndarray, crop: int, train: bool, rng: random.Random) -> np.ndarray:
    """Random (train) / centre (eval) crop + random horizontal mirror of a CHW image."""
    c, h, w = img.shape
    if crop and (h > crop or w > crop):
        if train:
            y0, x0 = rng.randint(0, h - crop), rng.randint(0, w - crop)
        else:
            y0, x0 = (h - crop) // 2, (w - crop) // 2
        img = img[:, y0:y0 + crop, x0:x0 + crop]
    if train and rng.random() < 0.5:
        img = img[:, :, ::-1]
    return np.ascontiguousarray(img)


class ImageBatchIter:
    """SINGA ``ImageBatchIter``: reads ``path label`` lines, decodes images
    with PIL in a background thread pool, applies ``transform(CHW uint8) ->
    float32 CHW`` and yields (images [B,C,H,W], labels [B])."""

    def __init__(self, list_file: str, batch_size: int, transform: Optional[Callable] = None, shuffle: bool = True,
                 image_folder: str = "", capacity: int = 4, workers: int = 2, seed: int = 0):
        self.items: List[Tuple[str, int]] = []
        with open(list_file) as f:
            for ln in f:
                p = ln.split()
                if len(p) >= 2:
                    self.items.append((os.path.join(image_folder, p[0]), int(p[1])))
        self.bs, self.shuffle, self.transform = batch_size, shuffle, transform
        self.rng = random.Random(seed)
        self.q: "queue.Queue" = queue.Queue(maxsize=capacity)
        self.workers = workers
        self.stop = threading.Event()
        self.thread = None

    def _load(self, path):
        from PIL import Image

        a = np.asarray(Image.open(path).convert("RGB"), dtype=np.uint8).transpose(2, 0, 1)
        return self.transform(a) if self.transform else a.astype(np.float32)

    def _run(self):
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(self.workers) as ex:
            while not self.stop.is_set():
                order = list(range(len(self.items)))
                if self.shuffle:
                    self.rng.shuffle(order)
                for b in range(len(order) // self.bs):
                    sel = [self.items[i] for i in order[b * self.bs:(b + 1) * self.bs]]
                    imgs = list(ex.map(lambda it: self._load(it[0]), sel))
                    self.q.put((np.stack(imgs), np.asarray([it[1] for it in sel], np.int32)))
                    if self.stop.is_set():
                        return

    def start(self):
        if self.thread is None:
            self.thread = threading.Thread(target=self._run, daemon=True)
            self.thread.start()
        return self

    def __iter__(self):
        return self.start()

    def __next__(self):
        return self.q.get()

    def end(self):
        self.stop.set()


class SyntheticImages:
    """Endless random (images, labels) of a fixed shape (benchmarks)."""

    def __init__(self, batch_size: int, shape: Sequence[int] = (3, 224, 224), num_classes: int = 1000, seed: int = 0,
                 fixed: bool = True):
        self.rng = np.random.RandomState(seed)
        self.bs, self.shape, self.k, self.fixed = batch_size, tuple(shape), num_classes, fixed
        self._cache = None

    def __iter__(self):
        return self

    def __next__(self):
        if self.fixed and self._cache is not None:
            return self._cache
        b = (self.rng.standard_normal((self.bs,) + self.shape).astype(np.float32),
             self.rng.randint(0, self.k, self.bs).astype(np.int32))
        if self.fixed:
            self._cache = b
        return b


class DevicePrefetcher:
    """Wrap a host iterator: batch i+1 is copied host->device on a side HIP
    stream (pinned staging) while batch i is being consumed."""

    def __init__(self, it, device: Optional[torch.device] = None):
        self.it = iter(it)
        self.device = device or torch.device("cuda")
        self.stream = _stream.pooled(self.device, "prefetch") if self.device.type == "cuda" else None
        self.next = None
        self._preload()

    def _preload(self):
        try:
            x, y = next(self.it)
        except StopIteration:
            self.next = None
            return
        if self.stream is None:
            self.next = (torch.as_tensor(x), torch.as_tensor(y))
            return
        xp, yp = torch.from_numpy(np.ascontiguousarray(x)).pin_memory(), torch.from_numpy(
            np.ascontiguousarray(y)).pin_memory()
        with self.stream:
            self.next = (xp.to(self.device, non_blocking=True), yp.to(self.device, non_blocking=True))

    def __iter__(self):
        return self

    def __next__(self):
        if self.next is None:
            raise StopIteration
        if self.stream is not None:
            _stream.Event().record(self.stream).wait()  # the consumer's stream joins the copies
        cur = self.next
        for t in cur:
            if self.stream is not None:
                _mem.record_stream(t, torch.cuda.current_stream(self.device))
        self._preload()
        return cur
