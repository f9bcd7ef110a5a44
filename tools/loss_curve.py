"""Print a model's training-loss curve on a fixed synthetic batch (sanity
checks of the optimisation dynamics; CPU or GPU)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--dropout", type=float, default=0.5)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    from singa_amd import device, opt, tensor
    from singa_amd.models import alexnet, mlp, resnet

    dev = device.get_default_device() if a.cpu else device.create_rocm_gpu()
    dev.SetRandSeed(0)
    dt = torch.float32 if a.fp32 else torch.bfloat16
    rng = np.random.RandomState(0)
    shape, ncls = (3, 224, 224), 1000
    if a.model == "alexnet":
        m = alexnet.create_model(num_classes=1000, dropout=a.dropout, compute_dtype=dt)
    elif a.model == "mlp":
        m, shape, ncls = mlp.deep_big_simple(), (784,), 10
    else:
        m = resnet.create_model(int(a.model.replace("resnet", "")), num_classes=1000, compute_dtype=dt)
    x = tensor.from_numpy(rng.standard_normal((a.batch,) + shape).astype(np.float32)).to_device(dev)
    y = tensor.from_numpy(rng.randint(0, ncls, a.batch).astype(np.int32)).to_device(dev)
    m.set_optimizer(opt.SGD(a.lr, a.momentum, weight_decay=5e-4))
    m.compile([x], is_train=True, use_graph=a.graph)
    m.train()
    ls = []
    for _ in range(a.steps):
        _, l = m(x, y)
        ls.append(round(float(l.data.float().cpu()), 4))
    print(json.dumps({"model": a.model, "batch": a.batch, "lr": a.lr, "dropout": a.dropout, "cpu": a.cpu,
                      "graph": a.graph, "loss": ls}))


if __name__ == "__main__":
    main()
