"""Debug: one downsampling Bottleneck, fused vs separate shortcut BN: per-parameter gradient differences."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import singa_amd  # noqa: E402
from singa_amd import autograd, device  # noqa: E402
from singa_amd.models.resnet import Bottleneck  # noqa: E402
from singa_amd.tensor import Tensor  # noqa: E402

singa_amd.set_deterministic(True)
res = {}
for fused in ("0", "1"):
    os.environ["SINGA_FUSED_DOWN_BN"] = fused
    dev = device.create_rocm_gpu()
    dev.SetRandSeed(1)
    blk = Bottleneck(16, 2, True)
    g = torch.Generator(device="cuda").manual_seed(2)
    xf = torch.randn(4, 64, 16, 16, device="cuda", generator=g)
    x = Tensor(data=xf.bfloat16().contiguous(memory_format=torch.channels_last), device=dev, requires_grad=True,
               stores_grad=False)
    autograd.training = True
    y = blk(x)
    dy = torch.randn(y.shape, device="cuda", generator=g)
    loss = autograd.reduce_sum(autograd.mul(y, Tensor(data=dy.bfloat16().contiguous(memory_format=torch.channels_last),
                                                      device=dev, requires_grad=False)), None)
    names = {id(p): k for k, p in blk.get_params().items()}
    grads = {names[id(p)]: gg.data.float().clone() for p, gg in autograd.backward(loss)}
    autograd.training = False
    res[fused] = (y.data.float().clone(), grads)
print("y equal:", torch.equal(res["0"][0], res["1"][0]))
for k in res["0"][1]:
    a, b = res["0"][1][k], res["1"][1].get(k)
    if b is None:
        print(k, "missing in fused")
        continue
    d = (a - b).abs().max().item()
    print(f"{k:16s} maxdiff {d:.3e}  norm {a.norm().item():.3e}  {'EQUAL' if torch.equal(a, b) else ''}")
