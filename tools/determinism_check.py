"""Run the same ResNet training-mode forward (and one step) several times from
the same weights and data; print the spread (a race or an uninitialised read
shows up as run-to-run differences far above fp32 atomic-order noise)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from singa_amd import autograd, device, opt, tensor  # noqa: E402
from singa_amd.models import resnet  # noqa: E402


def main():
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    hw = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    if os.environ.get("DET", "0") == "1":
        import singa_amd
        singa_amd.set_deterministic(True)
    dev = device.create_rocm_gpu()
    dev.SetRandSeed(0)
    rng = np.random.RandomState(0)
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    X = rng.randn(B, 3, hw, hw).astype(np.float32)
    Y = rng.randint(0, 10, B).astype(np.int32)
    m = resnet.create_model(depth, num_classes=10, compute_dtype=torch.bfloat16)
    m.set_optimizer(opt.SGD(0.005, 0.9))
    x, y = tensor.from_numpy(X, dev), tensor.from_numpy(Y, dev)
    m.compile([x], is_train=True)
    init = {k: v.data.clone() for k, v in m.get_states().items()}
    outs = []
    for rep in range(4):
        m.set_states(init)
        autograd.training = True
        o = m.forward(x)
        outs.append(o.data.float().clone())
        autograd.training = False
    for k in range(1, 4):
        print("train-mode forward rep", k, "max|diff|", float((outs[k] - outs[0]).abs().max()),
              "rel", float((outs[k] - outs[0]).norm() / outs[0].norm()))
    for name, mod in [("eval", False)]:
        autograd.training = False
        a = m.forward(x).data.float().clone()
        b = m.forward(x).data.float().clone()
        print(name, "forward rep max|diff|", float((a - b).abs().max()))


if __name__ == "__main__":
    main()
