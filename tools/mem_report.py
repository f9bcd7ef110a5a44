"""Memory footprint of the flagship step: the native pool's counters
(singa_amd.memory.stats) and PyTorch's allocator counters after a few
ResNet-50 training steps.

    python tools/mem_report.py [--batch 1024] [--steps 3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from singa_amd import device, memory, opt, tensor
    from singa_amd.models import resnet

    dev = device.create_rocm_gpu_on(0, set_default=True)
    m = resnet.create_model(50, num_classes=1000, compute_dtype=torch.bfloat16)
    m.set_optimizer(opt.SGD(0.01, 0.9, weight_decay=1e-4))
    rng = np.random.RandomState(0)
    x = tensor.from_numpy(rng.standard_normal((a.batch, 3, 224, 224)).astype(np.float32), dev)
    y = tensor.from_numpy(rng.randint(0, 1000, a.batch).astype(np.int32), dev)
    m.compile([x], is_train=True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        m(x, y)
    torch.cuda.synchronize()
    g = torch.device("cuda", 0)
    st = memory.stats(g)
    GiB = 2.0 ** 30
    print(f"native pool ({'on' if memory.enabled() else 'off'}): peak in use {st.get('peak_in_use_bytes', 0) / GiB:.2f} "
          f"GiB, reserved {st.get('reserved_bytes', 0) / GiB:.2f} GiB, driver allocs {st.get('driver_allocs', 0)}, "
          f"allocs {st.get('allocs', 0)}, hits {st.get('cache_hits', 0)}, live blocks {st.get('live_blocks', 0)}")
    print(f"torch allocator: peak allocated {torch.cuda.max_memory_allocated() / GiB:.2f} GiB, reserved "
          f"{torch.cuda.memory_reserved() / GiB:.2f} GiB, segments "
          f"{torch.cuda.memory_stats().get('segment.all.current', 0)}")
    print(f"{a.steps} steps in {time.perf_counter() - t0:.2f} s")


if __name__ == "__main__":
    main()
