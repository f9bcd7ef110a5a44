"""EASGD / RandomSync Worker workload for kernel-purity profiles: the
reference's mlp.conf MLP (784-2500-2000-1500-1000-500-10) trained by two
groups on ONE GPU -- two loopback ranks (threads, singa_amd.parallel.loop)
behind the real RcclCommunicator -- with the group exchange every
``--sync-frequency`` steps (overlapped on the comm stream for Elastic).

    python tools/easgd_workload.py [--ptype Elastic|RandomSync] [--steps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ptype", default="Elastic")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--sync-frequency", type=int, default=2)
    ap.add_argument("--ranks", type=int, default=2)
    a = ap.parse_args()
    from singa_amd import device
    from singa_amd.config import schema
    from singa_amd.parallel.loop import run_ranks
    from singa_amd.runtime import Worker

    text = open(os.path.join(os.path.dirname(__file__), "..", "examples", "mnist", "mlp.conf")).read()
    mp = schema.parse_text("ModelProto", text)
    mp.train_steps = a.steps
    mp.updater.param_type = a.ptype
    mp.updater.sync_frequency = a.sync_frequency
    mp.updater.warmup_steps = 2
    mp.display_frequency = max(1, a.steps // 2)
    mp.test_frequency = 0
    mp.validation_frequency = 0

    def rank(r, world, comm):
        w = Worker(mp, dev=device.create_rocm_gpu_on(0), comm=comm, log=lambda s: None, seed=r,
                   data_override={"*": {"shape": (28, 28), "nclass": 10, "seed": 3}})
        w.run()
        torch.cuda.current_stream().synchronize()
        return w.sync.nsync

    ns = run_ranks(rank, a.ranks, device=torch.device("cuda", 0), timeout_s=300.0)
    print(f"{a.ptype}: {a.ranks} loopback ranks, syncs per rank {ns}")


if __name__ == "__main__":
    main()
