"""Per-step workspace-arena hits/misses of a ResNet training step (eager
warm-up steps, then HIP-graph capture).  python tools/arena_check.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from singa_amd import device, opt, tensor  # noqa: E402
from singa_amd.models import resnet  # noqa: E402
from singa_amd.ops import functional as F  # noqa: E402

dev = device.create_rocm_gpu_on(0, set_default=True)
m = resnet.create_model(50, num_classes=1000, compute_dtype=torch.bfloat16)
m.set_optimizer(opt.SGD(lr=0.01, momentum=0.9))
x = tensor.from_numpy(np.random.randn(16, 3, 224, 224).astype(np.float32), dev)
y = tensor.from_numpy(np.random.randint(0, 1000, 16).astype(np.int32), dev)
m.compile([x], is_train=True, use_graph=True)
for i in range(5):
    m(x, y)
    torch.cuda.synchronize()
    a = F.ARENA
    print(f"step {i}: hits {a.hits} misses {a.misses} hwm {a.hwm} buf {None if a.buf is None else a.buf.numel()}",
          flush=True)
