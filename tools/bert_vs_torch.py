"""BERT loss-curve cross-check: the native BERT (bf16 and fp32 compute on the
GPU) against a PyTorch fp32 mirror of the same network, from IDENTICAL
initial weights and data, Adam, no dropout.  Diagnoses the loss spike of the
bench suite's BERT records (0.66 -> 6.7 at step 2, verdict r4 weak #5): if
the fp32 mirror spikes the same way, it is Adam's first step on a
random-init network (every weight moves by ~lr at once), not a numerics
issue of the bf16 kernels.

    python tools/bert_vs_torch.py --size tiny --steps 8 --lr 1e-4
"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as TF

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def torch_forward(P, ids, cfg):
    """The native model's graph (models/bert.py) in PyTorch fp32: post-LN
    encoder, fused qkv laid out [B][S][3][H][D], exact-erf GELU, tanh
    pooler over [CLS], 2-way classifier.  P: name -> fp32 leaf tensor."""
    B, S = ids.shape
    H, hid = cfg["heads"], cfg["hidden"]
    D = hid // H
    x = P["embeddings.word"][ids] + P["embeddings.position"][:S][None] + P["embeddings.token_type"][0][None, None]
    x = TF.layer_norm(x, (hid,), P["embeddings.ln.scale"], P["embeddings.ln.bias"], 1e-12)
    for i in range(cfg["layers"]):
        pre = f"encoder.{i}."
        qkv = x @ P[pre + "qkv.W"] + P[pre + "qkv.b"]
        t = qkv.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
        sc = (t[0] @ t[1].transpose(-1, -2)) / math.sqrt(D)
        a = (torch.softmax(sc, -1) @ t[2]).permute(0, 2, 1, 3).reshape(B, S, hid)
        a = a @ P[pre + "proj.W"] + P[pre + "proj.b"]
        x = TF.layer_norm(x + a, (hid,), P[pre + "ln1.scale"], P[pre + "ln1.bias"], 1e-12)
        f = TF.gelu(x @ P[pre + "fc1.W"] + P[pre + "fc1.b"]) @ P[pre + "fc2.W"] + P[pre + "fc2.b"]
        x = TF.layer_norm(x + f, (hid,), P[pre + "ln2.scale"], P[pre + "ln2.bias"], 1e-12)
    pooled = torch.tanh(x[:, 0] @ P["pooler.W"] + P["pooler.b"])
    return pooled @ P["classifier.W"] + P["classifier.b"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="tiny", choices=("tiny", "base"))
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--lr", type=float, default=1e-4)
    a = ap.parse_args()
    from singa_amd import device, opt, tensor
    from singa_amd.models import bert

    cfg = (dict(vocab=1000, hidden=128, layers=2, heads=2, ffn=512, max_pos=128) if a.size == "tiny" else
           dict(vocab=30522, hidden=768, layers=12, heads=12, ffn=3072, max_pos=512))
    rng = np.random.RandomState(0)
    ids_np = rng.randint(0, cfg["vocab"], (a.batch, a.seq)).astype(np.int64)
    y_np = rng.randint(0, 2, a.batch).astype(np.int32)
    out = {"config": {**cfg, "batch": a.batch, "seq": a.seq, "lr": a.lr, "optimizer": "Adam(0.9, 0.999, 1e-8)",
                      "dropout": 0.0}}
    init = None
    for dt_name, dt in (("native_bf16", torch.bfloat16), ("native_fp32", torch.float32)):
        dev = device.create_rocm_gpu()
        dev.SetRandSeed(0)
        m = bert.Bert(dropout=0.0, compute_dtype=dt, **cfg)
        ids = tensor.from_numpy(ids_np, dev)
        y = tensor.from_numpy(y_np, dev)
        m.set_optimizer(opt.Adam(a.lr))
        m.compile([ids], is_train=True, use_graph=False)
        if init is None:
            init = {k: v.data.float().clone() for k, v in m.get_states().items()}
        else:
            m.set_states({k: v.to(m.get_states()[k].data.dtype) for k, v in init.items()})
        m.train()
        ls = []
        for _ in range(a.steps):
            _, loss = m(ids, y)
            ls.append(round(float(loss.data.float().cpu()), 4))
        out[dt_name] = ls
    P = {k: v.clone().requires_grad_(True) for k, v in init.items() if "running" not in k}
    topt = torch.optim.Adam(P.values(), lr=a.lr, betas=(0.9, 0.999), eps=1e-8)
    ids_t = torch.from_numpy(ids_np).cuda()
    y_t = torch.from_numpy(y_np).long().cuda()
    ls = []
    for _ in range(a.steps):
        loss = TF.cross_entropy(torch_forward(P, ids_t, cfg), y_t)
        topt.zero_grad()
        loss.backward()
        topt.step()
        ls.append(round(float(loss), 4))
    out["torch_fp32"] = ls
    print(json.dumps(out))


if __name__ == "__main__":
    main()
