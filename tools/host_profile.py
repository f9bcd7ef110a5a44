"""Host-side cost of the flagship training step: how long the Python /
launch path takes to ENQUEUE one step (no synchronisation inside the loop)
next to the GPU time of the step, plus a cProfile of the enqueue path.

If enqueue time approaches the GPU step time the step is host-bound and
every microsecond of per-op Python overhead shows up in images/s.

    python tools/host_profile.py --steps 10 [--batch 1024] [--top 30]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    from singa_amd import device, opt, tensor
    from singa_amd.models import resnet

    dev = device.create_rocm_gpu_on(0, set_default=True)
    m = resnet.create_model(50, num_classes=1000, compute_dtype=torch.bfloat16)
    m.set_optimizer(opt.SGD(0.01, 0.9, weight_decay=1e-4))
    rng = np.random.RandomState(0)
    x = tensor.from_numpy(rng.standard_normal((a.batch, 3, 224, 224)).astype(np.float32), dev)
    y = tensor.from_numpy(rng.randint(0, 1000, a.batch).astype(np.int32), dev)
    m.compile([x], is_train=True, use_graph=False)
    for _ in range(3):
        m(x, y)
    torch.cuda.synchronize()
    enq = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s = time.perf_counter()
        m(x, y)
        enq.append(time.perf_counter() - s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    print(f"step wall {wall * 1e3:.2f} ms; host enqueue per step: mean {np.mean(enq) * 1e3:.2f} ms, "
          f"min {np.min(enq) * 1e3:.2f}, max {np.max(enq) * 1e3:.2f}")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        m(x, y)
    pr.disable()
    torch.cuda.synchronize()
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(a.top)
    print(out.getvalue())
    return 0


if __name__ == "__main__":
    sys.exit(main())
