"""Training-dynamics cross-check: singa_amd ResNet-50 (bf16, eager and
HIP-graph) vs the same network in PyTorch fp32 (tools/torch_resnet_ref.R50)
from IDENTICAL initial weights and data; prints the loss curves."""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from singa_amd import device, opt, tensor  # noqa: E402
from singa_amd.models import resnet  # noqa: E402
from tools.torch_resnet_ref import R50  # noqa: E402


def copy_into_torch(m, tm):
    p = {k: v.data.float() for k, v in m.get_states().items()}
    sd = {}
    sd["stem.0.weight"] = p["conv1.W"]
    for a, b in (("weight", "scale"), ("bias", "bias"), ("running_mean", "running_mean"), ("running_var", "running_var")):
        sd[f"stem.1.{a}"] = p[f"bn1.{b}"]
    for i in range(16):
        pre = f"blocks.{i}."
        for j in (1, 2, 3):
            sd[f"layers.{i}.c{j}.weight"] = p[pre + f"conv{j}.W"]
            for a, b in (("weight", "scale"), ("bias", "bias"), ("running_mean", "running_mean"),
                         ("running_var", "running_var")):
                sd[f"layers.{i}.b{j}.{a}"] = p[pre + f"bn{j}.{b}"]
        if pre + "down_conv.W" in p:
            sd[f"layers.{i}.down.0.weight"] = p[pre + "down_conv.W"]
            for a, b in (("weight", "scale"), ("bias", "bias"), ("running_mean", "running_mean"),
                         ("running_var", "running_var")):
                sd[f"layers.{i}.down.1.{a}"] = p[pre + f"down_bn.{b}"]
    sd["fc.weight"] = p["fc.W"].t()
    sd["fc.bias"] = p["fc.b"]
    missing = tm.load_state_dict({k: v.contiguous() for k, v in sd.items()}, strict=False)
    assert not missing.missing_keys or all("num_batches" in k for k in missing.missing_keys), missing


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--lr", type=float, default=0.02)
    ap.add_argument("--set-default", action="store_true", help="make the GPU the default device (as bench.py does)")
    ap.add_argument("--modes", default="eager,graph")
    ap.add_argument("--no-sync", action="store_true", help="do not read the loss between steps (async replays)")
    ap.add_argument("--torch", action="store_true", default=True)
    ap.add_argument("--no-torch", dest="torch", action="store_false")
    a = ap.parse_args()
    rng = np.random.RandomState(0)
    X = rng.standard_normal((a.batch, 3, 224, 224)).astype(np.float32)
    Y = rng.randint(0, 1000, a.batch).astype(np.int32)
    out = {}
    init = None
    for mode in a.modes.split(","):
        dev = device.create_rocm_gpu(set_default=a.set_default)
        dev.SetRandSeed(7)
        m = resnet.resnet50(num_classes=1000, compute_dtype=torch.bfloat16)
        m.set_optimizer(opt.SGD(a.lr, 0.9, weight_decay=1e-4))
        x, y = tensor.from_numpy(X, dev), tensor.from_numpy(Y, dev)
        m.compile([x], is_train=True, use_graph=(mode == "graph"))
        if init is None:
            init = {k: v.data.clone() for k, v in m.get_states().items()}
            tm = R50().cuda()
            copy_into_torch(m, tm)
        else:
            m.set_states(init)
        ls = []
        for _ in range(a.steps):
            _, l = m(x, y)
            ls.append(l.data.float().clone() if a.no_sync else round(float(l.data.float().cpu()), 4))
        out[mode] = [round(float(v), 4) for v in ls]
    if not a.torch:
        print(json.dumps(out))
        return
    topt = torch.optim.SGD(tm.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4)
    xt, yt = torch.from_numpy(X).cuda(), torch.from_numpy(Y).long().cuda()
    ls = []
    for _ in range(a.steps):
        loss = nn.functional.cross_entropy(tm(xt), yt)
        topt.zero_grad()
        loss.backward()
        topt.step()
        ls.append(round(float(loss), 4))
    out["torch_fp32"] = ls
    print(json.dumps(out))


if __name__ == "__main__":
    main()
