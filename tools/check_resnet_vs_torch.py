"""Training-dynamics cross-check: singa_amd ResNet-50 (bf16, eager and
HIP-graph) vs the same network in PyTorch fp32 (tools/torch_resnet_ref.R50)
from IDENTICAL initial weights and data; prints the loss curves.

``--gamma3 v`` initialises the last BN scale of every bottleneck to v in both
networks (Goyal et al.'s zero-gamma init at v = 0): each residual branch then
starts (near) the identity, which takes the network out of the chaotic regime
of a random-init ResNet-50 -- where a 2^-9 perturbation of the input alone
moves the step-1 gradients by O(1) -- so a per-parameter gradient comparison
can detect a kernel error.  ``--dtype fp32`` runs our network on the
exact-f32 MFMA kernels instead of bf16."""
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


def name_map(m):
    """our parameter name -> the torch R50 parameter name (as copy_into_torch)."""
    mp = {"conv1.W": "stem.0.weight", "bn1.scale": "stem.1.weight", "bn1.bias": "stem.1.bias",
          "fc.W": "fc.weight", "fc.b": "fc.bias"}
    for i in range(16):
        pre = f"blocks.{i}."
        for j in (1, 2, 3):
            mp[pre + f"conv{j}.W"] = f"layers.{i}.c{j}.weight"
            mp[pre + f"bn{j}.scale"] = f"layers.{i}.b{j}.weight"
            mp[pre + f"bn{j}.bias"] = f"layers.{i}.b{j}.bias"
        mp[pre + "down_conv.W"] = f"layers.{i}.down.0.weight"
        mp[pre + "down_bn.scale"] = f"layers.{i}.down.1.weight"
        mp[pre + "down_bn.bias"] = f"layers.{i}.down.1.bias"
    return mp


def step1_grads(m, x, y):
    """One forward + backward of our model (no update): name -> fp32 gradient
    in the logical (torch) layout."""
    from singa_amd import autograd

    # the parameters' gradients accumulate into the optimizer's flat buffer,
    # which a training step zeroes first (Optimizer.backward_and_update):
    # zero it here too, or the yielded views hold stale contents plus this pass
    st = getattr(m.optimizer, "store", None)
    if st is not None:
        st.zero_grad()
    autograd.training = True
    try:
        out = m.forward(x)
        loss = m.loss_fn(out, y)
        g = {}
        for p, gg in autograd.backward(loss):
            torch.cuda.synchronize()  # (side-stream work complete before the copy)
            g[id(p)] = gg.data.float().clone()
        torch.cuda.synchronize()
    finally:
        autograd.training = False
    res = {}
    for k, p in m.get_params().items():
        if id(p) in g:
            t = g[id(p)]
            res[k] = t.reshape(p.data.shape) if t.numel() == p.data.numel() else t
    return res


def _summary(errs):
    v = sorted(errs.values())
    return {"n": len(v), "max": max(v), "median": v[len(v) // 2],
            "worst5": sorted(errs.items(), key=lambda kv: -kv[1])[:5], "per_param": errs}


def grad_report(m, tm, x, y, xt, yt):
    """Step-1 gradient of every parameter against PyTorch fp32, and -- the
    yardstick -- PyTorch's own bf16 autocast run against the same fp32
    gradients: at random init a deep BN/ReLU network is chaotic (a rounding
    perturbation grows layer by layer backwards), so the bf16-vs-fp32 distance
    of the early layers' gradients is a property of the network, not of a
    kernel; ours should sit at PyTorch bf16's own distance."""
    import copy

    ours = step1_grads(m, x, y)
    tb = copy.deepcopy(tm)
    state = {k: v.clone() for k, v in tm.state_dict().items()}
    tm.zero_grad()
    nn.functional.cross_entropy(tm(xt), yt).backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lb = nn.functional.cross_entropy(tb(xt), yt)
    lb.backward()
    # the chaos yardstick proper: the SAME fp32 network, only its input
    # rounded to bf16 (a 2^-9 relative perturbation of one tensor)
    tr = copy.deepcopy(tm)
    tr.load_state_dict(state)
    tr.zero_grad()
    nn.functional.cross_entropy(tr(xt.bfloat16().float()), yt).backward()
    # the fp32 floor: the same fp32 network with its input moved by ONE fp32
    # ulp (x * (1 + 2^-23)) -- what any change of fp32 summation order does
    tu = copy.deepcopy(tm)
    tu.load_state_dict(state)
    tu.zero_grad()
    nn.functional.cross_entropy(tu(xt * (1.0 + 2.0 ** -23)), yt).backward()
    tm.load_state_dict(state)  # (the running statistics the forwards moved)
    tp, tq, tz = dict(tm.named_parameters()), dict(tb.named_parameters()), dict(tr.named_parameters())
    tw = dict(tu.named_parameters())
    errs, errs_tb, errs_in, errs_ulp = {}, {}, {}, {}
    zero = []  # parameters whose reference gradient is exactly zero (zero-gamma branches): ours must be too
    rel = lambda u, v: float((u - v).norm() / (v.norm() + 1e-30))  # noqa: E731
    for k, tn in name_map(m).items():
        if k not in ours or tn not in tp:
            continue
        a, b, c, d = ours[k].float(), tp[tn].grad.float(), tq[tn].grad.float(), tz[tn].grad.float()
        e = tw[tn].grad.float()
        if k == "fc.W":
            b, c, d, e = b.t(), c.t(), d.t(), e.t()
        a = a.reshape(b.shape)
        if float(b.norm()) == 0.0:
            zero.append((k, float(a.norm())))
            continue
        errs[k], errs_tb[k], errs_in[k], errs_ulp[k] = rel(a, b), rel(c, b), rel(d, b), rel(e, b)
    return {"ours_vs_torch_fp32": _summary(errs), "torch_bf16_autocast_vs_torch_fp32": _summary(errs_tb),
            "torch_fp32_bf16_rounded_input_vs_torch_fp32": _summary(errs_in),
            "torch_fp32_one_ulp_input_vs_torch_fp32": _summary(errs_ulp),
            "zero_reference_grads": {"n": len(zero), "ours_max_norm": max([z for _, z in zero], default=0.0)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grads", action="store_true", help="also compare the step-1 gradient of every parameter")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--lr", type=float, default=0.02)
    ap.add_argument("--set-default", action="store_true", help="make the GPU the default device (as bench.py does)")
    ap.add_argument("--modes", default="eager,graph")
    ap.add_argument("--no-sync", action="store_true", help="do not read the loss between steps (async replays)")
    ap.add_argument("--torch", action="store_true", default=True)
    ap.add_argument("--no-torch", dest="torch", action="store_false")
    ap.add_argument("--gamma3", type=float, default=None,
                    help="initial scale of every bottleneck's last BN (both networks); 0 = zero-gamma init")
    ap.add_argument("--dtype", choices=("bf16", "fp32"), default="bf16", help="our compute dtype")
    ap.add_argument("--out", default="", help="also write the JSON record here")
    a = ap.parse_args()
    rng = np.random.RandomState(0)
    X = rng.standard_normal((a.batch, 3, 224, 224)).astype(np.float32)
    Y = rng.randint(0, 1000, a.batch).astype(np.int32)
    out = {}
    init = None
    for mode in a.modes.split(","):
        dev = device.create_rocm_gpu(set_default=a.set_default)
        dev.SetRandSeed(7)
        m = resnet.resnet50(num_classes=1000,
                            compute_dtype=torch.bfloat16 if a.dtype == "bf16" else torch.float32)
        m.set_optimizer(opt.SGD(a.lr, 0.9, weight_decay=1e-4))
        x, y = tensor.from_numpy(X, dev), tensor.from_numpy(Y, dev)
        m.compile([x], is_train=True, use_graph=(mode == "graph"))
        if init is None and a.gamma3 is not None:
            from singa_amd.ops import glue as G
            for b in m.blocks:
                G.fill_(b.bn3.scale.data, a.gamma3)
            torch.cuda.synchronize()
        if init is None:
            init = {k: v.data.clone() for k, v in m.get_states().items()}
            tm = R50().cuda()
            copy_into_torch(m, tm)
            if a.grads:
                xt0, yt0 = torch.from_numpy(X).cuda(), torch.from_numpy(Y).long().cuda()
                out["grads_step1"] = grad_report(m, tm, x, y, xt0, yt0)
                m.set_states(init)
        else:
            m.set_states(init)
        ls = []
        for _ in range(a.steps):
            _, l = m(x, y)
            ls.append(l.data.float().clone() if a.no_sync else round(float(l.data.float().cpu()), 4))
        out[mode] = [round(float(v), 4) for v in ls]
    out["config"] = {"batch": a.batch, "steps": a.steps, "lr": a.lr, "gamma3": a.gamma3, "dtype": a.dtype,
                     "modes": a.modes}
    if not a.torch:
        _emit(out, a.out)
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
    for mode in a.modes.split(","):
        if mode in out:
            d = [abs(u - v) / max(abs(v), 1e-12) for u, v in zip(out[mode], ls)]
            out[f"loss_rel_diff_{mode}_max"] = round(max(d), 5)
    _emit(out, a.out)


def _emit(out, path):
    line = json.dumps(out)
    print(line)
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
