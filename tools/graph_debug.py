"""Diagnose HIP-graph replay divergence: run the bench flow and record, after
every call, the loss, the flat-weight norm, the momentum norm and hp (device)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=8)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--read", default="", help="comma list of call indices after which to read the loss (sync)")
    a = ap.parse_args()
    from singa_amd import device, opt, tensor
    from singa_amd.models import resnet
    dev = device.create_rocm_gpu_on(0, set_default=True)
    dev.SetRandSeed(1234)
    m = resnet.create_model(50, num_classes=1000, compute_dtype=torch.bfloat16)
    sgd = opt.SGD(lr=0.01, momentum=0.9, weight_decay=1e-4)
    m.set_optimizer(sgd)
    rng = np.random.RandomState(0)
    x = rng.standard_normal((a.batch, 3, 224, 224)).astype(np.float32)
    y = rng.randint(0, 1000, size=(a.batch,)).astype(np.int32)
    tx, ty = tensor.from_numpy(x, dev), tensor.from_numpy(y, dev)
    m.compile([tx], is_train=True, use_graph=True)
    st = sgd.store
    reads = {int(v) for v in a.read.split(",") if v}
    rec = []
    for i in range(a.calls):
        out, loss = m(tx, ty)
        rec.append((loss.data.float().clone(), st.w.norm().clone(), st.s1.norm().clone(), sgd._hp_dev.clone(),
                    st.g.norm().clone()))
        if i in reads:
            float(loss.data.float().item())
    torch.cuda.synchronize()
    for i, (l, w, s1, hp, g) in enumerate(rec):
        print(json.dumps({"call": i + 1, "loss": float(l), "w": float(w), "mom": float(s1), "g": float(g),
                          "hp": [float(v) for v in hp.cpu()]}))


if __name__ == "__main__":
    main()
