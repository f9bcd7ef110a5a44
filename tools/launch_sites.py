"""Which Python lines launch a training step's kernels: one eager ResNet-50
step (after warm-up) with SG_LAUNCH_TRACE=1 (ops/native.py), every binding
call counted by (binding, call site, caller).

    SG_LAUNCH_TRACE=1 python tools/launch_sites.py [--batch 64] [--model resnet50]
"""
import argparse
import os
import sys

os.environ["SG_LAUNCH_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--top", type=int, default=80)
    a = ap.parse_args()
    from singa_amd import device, opt, tensor
    from singa_amd.models import resnet
    from singa_amd.ops import native as N

    dev = device.create_rocm_gpu_on(0, set_default=True)
    m = resnet.create_model(50, num_classes=1000, compute_dtype=torch.bfloat16)
    m.set_optimizer(opt.SGD(0.01, 0.9, weight_decay=1e-4))
    rng = np.random.RandomState(0)
    x = tensor.from_numpy(rng.standard_normal((a.batch, 3, 224, 224)).astype(np.float32), dev)
    y = tensor.from_numpy(rng.randint(0, 1000, a.batch).astype(np.int32), dev)
    m.compile([x], is_train=True, use_graph=False)
    m.train()
    for _ in range(2):
        m(x, y)
    torch.cuda.synchronize()
    L = N.lib()
    L.enabled = True
    m(x, y)
    torch.cuda.synchronize()
    L.enabled = False
    tot = sum(L.counts.values())
    byname = {}
    for (k, site), c in L.counts.items():
        byname[k] = byname.get(k, 0) + c
    print(f"# {tot} binding calls in one step")
    for k, c in sorted(byname.items(), key=lambda kv: -kv[1]):
        print(f"{c:6d}  {k}")
    print("# by call site")
    for (k, site), c in L.counts.most_common(a.top):
        print(f"{c:6d}  {k:28s} {site}")


if __name__ == "__main__":
    main()
