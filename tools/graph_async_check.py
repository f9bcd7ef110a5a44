"""Reproducer for divergence of asynchronously replayed training graphs:
runs ``trials`` fresh models x (warmup + steps) with no host sync inside the
loop, records every loss on the device, and reports which trials blew up and
which parameters hold non-finite / huge values afterwards."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mlp")
    ap.add_argument("--trials", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--sync_every", type=int, default=0)
    ap.add_argument("--mid_sync", type=int, default=1, help="synchronize between warmup and timed steps")
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    from singa_amd import device, opt, tensor
    from singa_amd.models import alexnet, mlp

    dev = device.create_rocm_gpu()
    rng = np.random.RandomState(0)
    for t in range(a.trials):
        dev.SetRandSeed(0)
        if a.model == "mlp":
            m, shape, ncls = mlp.deep_big_simple(), (784,), 10
            o = opt.SGD(0.001, 0.9)
        else:
            m, shape, ncls = alexnet.create_model(compute_dtype=torch.bfloat16), (3, 224, 224), 1000
            o = opt.SGD(0.01, 0.9, weight_decay=5e-4)
        x = tensor.from_numpy(rng.rand(a.batch, *shape).astype(np.float32)).to_device(dev)
        y = tensor.from_numpy(rng.randint(0, ncls, a.batch).astype(np.int32)).to_device(dev)
        m.set_optimizer(o)
        m.compile([x], is_train=True, use_graph=bool(a.graph))
        m.train()
        curve = []
        for i in range(a.warmup + a.steps):
            if i == a.warmup and a.mid_sync:
                torch.cuda.synchronize()
            _, l = m(x, y)
            curve.append(l.data.detach().float().reshape(()).clone())
            if a.sync_every and (i + 1) % a.sync_every == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        c = [float(v) for v in curve]
        bad = [i for i, v in enumerate(c) if not np.isfinite(v) or v > 50]
        st = o.store
        info = []
        if bad:
            for p, off in zip(st.params, st.offsets):
                n = p.data.numel()
                w = st.w[off:off + n]
                s1 = st.s1[off:off + n]
                g = st.g[off:off + n]
                info.append((p.name, tuple(p.data.shape), float(w.abs().max()), float(s1.abs().max()),
                             float(g.abs().max())))
        print(json.dumps({"trial": t, "graph": a.graph, "sync_every": a.sync_every, "first_bad": bad[0] if bad else None,
                          "curve": [round(v, 4) for v in c[:10]], "params": info}), flush=True)
        del m, o, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
