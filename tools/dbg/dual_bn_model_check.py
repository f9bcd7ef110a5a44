"""Debug: ResNet-18 one training step, fused vs separate shortcut BN: which states differ."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import singa_amd  # noqa: E402
from singa_amd import device, opt, tensor  # noqa: E402
from singa_amd.models import resnet  # noqa: E402

singa_amd.set_deterministic(True)
rng = np.random.RandomState(2)
X = rng.randn(8, 3, 64, 64).astype(np.float32)
Y = rng.randint(0, 10, 8).astype(np.int32)
init, out = None, {}
for fused in ("0", "1"):
    os.environ["SINGA_FUSED_DOWN_BN"] = fused
    dev = device.create_rocm_gpu()
    dev.SetRandSeed(0)
    m = resnet.create_model(int(sys.argv[1]) if len(sys.argv) > 1 else 18, num_classes=10,
                            compute_dtype=torch.bfloat16)
    m.set_optimizer(opt.SGD(0.005, 0.9, weight_decay=1e-4))
    x = tensor.from_numpy(X, dev)
    y = tensor.from_numpy(Y, dev)
    m.compile([x], is_train=True, use_graph=False)
    if init is None:
        init = {k: v.data.clone() for k, v in m.get_states().items()}
    else:
        m.set_states(init)
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ls = []
    for _ in range(steps):
        _, l = m(x, y)
        ls.append(float(l.data.float().cpu()))
    out[fused] = (ls, {k: v.data.float().clone() for k, v in m.get_states().items()})
print("loss", out["0"][0], out["1"][0])
for k in out["0"][1]:
    a, b = out["0"][1][k], out["1"][1][k]
    if not torch.equal(a, b):
        d0 = (a - init[k].float()).abs().max().item()
        print(f"{k:40s} maxdiff {(a - b).abs().max().item():.3e}  step-update {d0:.3e}")
