"""Debug: a 3-bottleneck chain (stride-1 down, stride-2 down, identity) in
three modes -- unfused, fused tails with the compact strided shortcut
gradient, fused tails with it placed eagerly -- against PyTorch fp32
(tools/torch_resnet_ref Bottleneck blocks with copied weights)."""
import json
import os
import sys

import torch
import torch.nn.functional as TF

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-30))


def main():
    from singa_amd import autograd as AG
    from singa_amd import device
    from singa_amd.models.resnet import Bottleneck
    from singa_amd.ops import functional as FF
    from singa_amd.tensor import Tensor

    gpu = torch.device("cuda")
    cl = lambda t: t.contiguous(memory_format=torch.channels_last)  # noqa: E731
    dev = device.create_rocm_gpu()
    dev.SetRandSeed(13)
    blks = [Bottleneck(64, 1, True), Bottleneck(64, 2, True), Bottleneck(64, 1, False)]
    g0 = torch.Generator(device=gpu).manual_seed(6)
    xf = torch.randn(8, 128, 28, 28, device=gpu, generator=g0)
    dyt = None

    def run(on, lazy):
        nonlocal dyt
        on0, lz0 = FF.BNRES, FF.STRIDED_LAZY
        FF.BNRES, FF.STRIDED_LAZY = on, lazy
        AG.training = True
        try:
            x = Tensor(data=cl(xf).bfloat16(), device=dev, requires_grad=True, stores_grad=False)
            h = x
            outs = []
            for b in blks:
                h = b(h)
                outs.append(h.data.float().clone())
            if dyt is None:
                dyt = (torch.rand(h.shape, device=gpu, generator=g0) + 0.5 if os.environ.get("DBG_POS") else
                       torch.randn(h.shape, device=gpu, generator=g0))
            loss_t = AG.reduce_sum(AG.mul(h, Tensor(data=cl(dyt).bfloat16(), device=dev, requires_grad=False)), None)
            gr = {id(p): gg.data.float().clone() for p, gg in AG.backward(loss_t)}
        finally:
            AG.training = False
            FF.BNRES, FF.STRIDED_LAZY = on0, lz0
        return outs, gr

    res = {"off": run(False, True), "on_lazy": run(True, True), "on_place": run(True, False)}

    # fp32 torch reference with the same weights (batch-stat BN, training mode)
    def tblock(b, x):
        def bn(t, layer, relu):
            y = TF.batch_norm(t, None, None, layer.scale.data.float(), layer.bias.data.float(), True, 0.0, layer.eps)
            return torch.relu(y) if relu else y
        o = bn(TF.conv2d(x, b.conv1.W.data.float()), b.bn1, True)
        o = bn(TF.conv2d(o, b.conv2.W.data.float(), stride=b.conv2.stride, padding=1), b.bn2, True)
        o = bn(TF.conv2d(o, b.conv3.W.data.float()), b.bn3, False)
        if b.has_down:
            sc = bn(TF.conv2d(x, b.down_conv.W.data.float(), stride=b.down_conv.stride), b.down_bn, False)
        else:
            sc = x
        return torch.relu(o + sc)
    params = [(f"{i}.{k}", p) for i, b in enumerate(blks) for k, p in b.get_params().items()]
    leaves = {n: p.data.float().clone().requires_grad_(True) for n, p in params}
    saved = {n: p.data for n, p in params}
    for n, p in params:
        p.data = leaves[n]
    try:
        h = xf.bfloat16().float()
        touts = []
        for b in blks:
            h = tblock(b, h)
            touts.append(h.detach())
        (h * cl(dyt).bfloat16().float()).sum().backward()
    finally:
        for n, p in params:
            p.data = saved[n]
    tg = {n: leaves[n].grad for n, _ in params}
    for mode, (outs, gr) in res.items():
        fo = [round(rel(o, t), 4) for o, t in zip(outs, touts)]
        ge = {n: rel(gr[id(p)], tg[n]) for n, p in params}
        worst = sorted(ge.items(), key=lambda kv: -kv[1])[:4]
        print(json.dumps({"mode": mode, "fwd_rel": fo, "grad_max": round(max(ge.values()), 4),
                          "grad_median": round(sorted(ge.values())[len(ge) // 2], 4),
                          "worst": [(k, round(v, 4)) for k, v in worst]}), flush=True)
    for a, b in (("on_lazy", "on_place"), ("on_lazy", "off"), ("on_place", "off")):
        d = max(rel(res[a][1][id(p)], res[b][1][id(p)]) for _, p in params)
        print(json.dumps({"pair": [a, b], "grad_max_rel": round(d, 4),
                          "fwd": [round(rel(x, y), 4) for x, y in zip(res[a][0], res[b][0])]}))


if __name__ == "__main__":
    main()
