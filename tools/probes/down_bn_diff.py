"""Fused vs unfused shortcut BN (DualBNAddReLU) for one downsampling
Bottleneck: per-gradient max |diff| and magnitude (diagnostic for
tests/test_models_gpu.py::test_fused_downsample_bn_block_bitwise)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import singa_amd  # noqa: E402
from singa_amd import autograd as AG, device  # noqa: E402
from singa_amd.models.resnet import Bottleneck  # noqa: E402
from singa_amd.tensor import Tensor  # noqa: E402

stride = int(sys.argv[1]) if len(sys.argv) > 1 else 2
gpu = torch.device("cuda", 0)
singa_amd.set_deterministic(True)
res = {}
for fused in ("0", "1"):
    os.environ["SINGA_FUSED_DOWN_BN"] = fused
    dev = device.create_rocm_gpu()
    dev.SetRandSeed(1)
    blk = Bottleneck(16, stride, True)
    g = torch.Generator(device=gpu).manual_seed(2)
    xf = torch.randn(4, 64, 16, 16, device=gpu, generator=g)
    x = Tensor(data=xf.bfloat16().contiguous(memory_format=torch.channels_last), device=dev, requires_grad=True,
               stores_grad=True)
    AG.training = True
    y = blk(x)
    dy = torch.randn(y.shape, device=gpu, generator=g)
    loss = AG.reduce_sum(AG.mul(y, Tensor(data=dy.bfloat16().contiguous(memory_format=torch.channels_last),
                                          device=dev, requires_grad=False)), None)
    names = {id(p): k for k, p in blk.get_params().items()}
    names[id(x)] = "x"
    grads = {names[id(p)]: gg.data.float().clone() for p, gg in AG.backward(loss)}
    AG.training = False
    res[fused] = grads
for k in res["0"]:
    a, b = res["0"][k], res["1"][k]
    print(f"{k:16s} max|a| {float(a.abs().max()):10.4f}  max|diff| {float((a - b).abs().max()):.3e}  "
          f"ndiff {int((a != b).sum())}/{a.numel()}")
