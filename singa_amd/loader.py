"""``loader`` tool (reference C28, tools/data_loader/data_loader.cc): build
Shards from raw datasets, or split a shard.

    python -m singa_amd.loader --datasource mnist --imagefile train-images-idx3-ubyte \\
        --labelfile train-labels-idx1-ubyte --shard_folder /data/mnist/train
    python -m singa_amd.loader --datasource imagenet --shard_folder /data/in1k \\
        --mean mean.binaryproto --width 256 --height 256      # reads <folder>/rid.txt, <folder>/img/
    python -m singa_amd.loader --input /data/mnist/train --mode equal --n 4 --prefix /data/mnist/part
    python -m singa_amd.loader --input /data/mnist/train --mode first --n 50000 --prefix /data/mnist/tv

MNIST conversion and splitting are native (``_core.load_mnist``,
``split_shard``, ``split_shard_n``).  ImageNet images are decoded/resized
with PIL (the reference used OpenCV) and stored CHW as ``pixel - mean``
bytes like data_source.cc:150-183; the per-pixel mean is a ``BlobProto``
binary file (read with protobuf, no code execution), or omitted.
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import Optional

import numpy as np


def _core():
    from . import _core as C

    return C


def load_mnist(imagefile: str, labelfile: str, shard_folder: str, limit: int = 0) -> int:
    return int(_core().load_mnist(imagefile, labelfile, shard_folder, limit))


def split(num: int, input: str, prefix: str):
    return list(_core().split_shard(num, input, prefix))


def split_n(n: int, input: str, prefix: str):
    return list(_core().split_shard_n(n, input, prefix))


def read_mean(path: str) -> Optional[np.ndarray]:
    """BlobProto (num, channels, height, width, data) -> float32 [C,H,W]."""
    if not path or not os.path.exists(path):
        return None
    from .config import schema

    bp = schema.new("BlobProto")
    with open(path, "rb") as f:
        bp.ParseFromString(f.read())
    a = np.asarray(bp.data, dtype=np.float32)
    c, h, w = max(1, bp.channels), max(1, bp.height), max(1, bp.width)
    return a[:c * h * w].reshape(c, h, w)


def write_mean(path: str, mean: np.ndarray) -> None:
    from .config import schema

    bp = schema.new("BlobProto")
    c, h, w = mean.shape
    bp.num, bp.channels, bp.height, bp.width = 1, c, h, w
    bp.data.extend(mean.reshape(-1).astype(np.float32).tolist())
    with open(path, "wb") as f:
        f.write(bp.SerializeToString())


def load_imagenet(folder: str, meanfile: Optional[str], width: int, height: int,
                  shard_folder: Optional[str] = None, limit: int = 0) -> int:
    from PIL import Image

    C = _core()
    mean = read_mean(meanfile) if meanfile else None
    out = shard_folder or folder
    os.makedirs(out, exist_ok=True)
    shard = C.Shard(out, 2)  # kAppend
    lines = []
    with open(os.path.join(folder, "rid.txt")) as f:
        for ln in f:
            parts = ln.split()
            if len(parts) >= 2:
                lines.append((parts[0], int(parts[1])))
    if limit:
        lines = lines[:limit]
    n = 0
    for key, label in lines:
        try:
            im = Image.open(os.path.join(folder, "img", key)).convert("RGB")
        except OSError:
            print(f"invalid img {key}", file=sys.stderr)
            continue
        if width > 0 and height > 0:
            im = im.resize((width, height), Image.BILINEAR)
        chw = np.asarray(im, dtype=np.float32).transpose(2, 0, 1)
        if mean is not None:
            chw = chw - mean[:, :chw.shape[1], :chw.shape[2]]
        pix = np.clip(np.rint(chw), -128, 255).astype(np.int16).astype(np.uint8).tobytes()
        rec = C.encode_record([3, chw.shape[1], chw.shape[2]], int(label), pix, [])
        if shard.insert(key.encode(), rec):
            n += 1
    shard.flush()
    return n


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="loader", description=__doc__.split("\n\n")[0])
    ap.add_argument("--datasource", default="mnist")
    ap.add_argument("--imagefile", default="train-images-idx3-ubyte")
    ap.add_argument("--labelfile", default="train-labels-idx1-ubyte")
    ap.add_argument("--shard_folder", default="shard")
    ap.add_argument("--mean", default="")
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--mode", default="equal", help="equal: SplitN; otherwise Split(first n)")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--input", default="")
    ap.add_argument("--prefix", default="")
    ap.add_argument("--limit", type=int, default=0, help="convert at most this many records")
    a = ap.parse_args(argv)
    if a.input:
        counts = split_n(a.n, a.input, a.prefix) if a.mode == "equal" else split(a.n, a.input, a.prefix)
        for i, c in enumerate(counts):
            print(f"{c} records are inserted into {a.prefix}-{i}")
        return 0
    if a.datasource == "mnist":
        n = load_mnist(a.imagefile, a.labelfile, a.shard_folder, a.limit)
    else:
        n = load_imagenet(a.shard_folder, a.mean, a.width, a.height, limit=a.limit)
    print(f"inserted {n} records into {a.shard_folder}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
