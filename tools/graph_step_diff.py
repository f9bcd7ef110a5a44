"""Per-step, per-parameter comparison of graph-replayed vs eager training
(weights snapshotted on the device after every step, no host sync in the
loop except an optional one between warmup and timed steps)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def run(graph, mid_sync, a):
    from singa_amd import device, opt, tensor
    from singa_amd.models import mlp

    dev = device.create_rocm_gpu()
    dev.SetRandSeed(0)
    rng = np.random.RandomState(0)
    m = mlp.deep_big_simple()
    o = opt.SGD(0.001, 0.9)
    x = tensor.from_numpy(rng.rand(a.batch, 784).astype(np.float32)).to_device(dev)
    y = tensor.from_numpy(rng.randint(0, 10, a.batch).astype(np.int32)).to_device(dev)
    m.set_optimizer(o)
    m.compile([x], is_train=True, use_graph=graph)
    m.train()
    snaps, gs, losses = [], [], []
    for i in range(a.steps):
        if i == a.warmup and mid_sync:
            torch.cuda.synchronize()
        _, l = m(x, y)
        snaps.append(o.store.w.clone())
        gs.append(o.store.g.clone())
        losses.append(l.data.detach().float().reshape(()).clone())
    torch.cuda.synchronize()
    return o.store, snaps, gs, [float(v) for v in losses]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=9)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    st, we, ge, le = run(False, False, a)
    _, wg, gg, lg = run(True, True, a)
    print("eager loss", [round(v, 4) for v in le])
    print("graph loss", [round(v, 4) for v in lg])
    for i in range(a.steps):
        row = []
        for p, off in zip(st.params, st.offsets):
            n = p.data.numel()
            dw = float((we[i][off:off + n] - wg[i][off:off + n]).abs().max())
            dg = float((ge[i][off:off + n] - gg[i][off:off + n]).abs().max())
            row.append(f"{p.name}:w{dw:.1e}/g{dg:.1e}")
        print(i, " ".join(row))


if __name__ == "__main__":
    main()
