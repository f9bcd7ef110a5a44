"""Which parameters got no (or a non-finite) gradient after a few ResNet-50
training steps (bench.py's dead-gradient guard, per parameter name)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from singa_amd import device, opt, tensor
    from singa_amd.models import resnet
    from singa_amd.ops import glue as G
    from singa_amd.parallel import DistOpt, init_distributed

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = device.create_rocm_gpu_on(0, set_default=True)
    dev.SetRandSeed(1234)
    comm = init_distributed(rank=0, world_size=1, local_rank=0)
    m = resnet.create_model(50, num_classes=1000, compute_dtype=torch.bfloat16)
    optimizer = DistOpt(opt.SGD(lr=0.01, momentum=0.9, weight_decay=1e-4), comm=comm)
    m.set_optimizer(optimizer)
    rng = np.random.RandomState(0)
    tx = tensor.from_numpy(rng.standard_normal((B, 3, 224, 224)).astype(np.float32), dev)
    ty = tensor.from_numpy(rng.randint(0, 1000, size=(B,)).astype(np.int32), dev)
    m.compile([tx], is_train=True, use_graph=False)
    m.train()
    names = {id(p): k for k, p in m.get_params().items()}
    nosync = os.environ.get("DEAD_NOSYNC", "0") == "1"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for step in range(steps):
        m(tx, ty)
        if nosync and step + 1 < steps:
            continue  # back-to-back steps as bench.py's warmup (no host sync in between)
        torch.cuda.synchronize()
        st = optimizer.store
        norms = G.cat([G.reduce(st.g[off:off + p.data.numel()], None, "sumsq").reshape(1)
                       for p, off in zip(st.params, st.offsets)]).cpu()
        bad = [(names.get(id(p), "?"), float(norms[i])) for i, p in enumerate(st.params)
               if not (float(norms[i]) > 0.0 and np.isfinite(float(norms[i])))]
        print(f"step {step}: {len(bad)} bad of {len(st.params)}: {bad}", flush=True)


if __name__ == "__main__":
    main()
