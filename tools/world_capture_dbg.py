"""Step-by-step trace of the captured loopback world (diagnostics)."""
import faulthandler
import os
import sys
import threading

faulthandler.enable(all_threads=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def log(*a):
    print(f"[{threading.current_thread().name}]", *a, file=sys.stderr, flush=True)


def rank_fn(rank, world, comm, steps):
    from singa_amd import device, opt, tensor
    from singa_amd.models import mlp
    from singa_amd.parallel import DistOpt

    dev = device.create_rocm_gpu_on(0)
    rng = np.random.RandomState(0)
    x = tensor.from_numpy(rng.randn(16, 40).astype(np.float32), dev)
    y = tensor.from_numpy(rng.randint(0, 10, 16).astype(np.int32), dev)
    m = mlp.create_model((64, 48), 10)
    m.compile([x], is_train=False)
    log("built")
    m.set_optimizer(DistOpt(opt.SGD(0.1, 0.9), comm=comm, bucket_mb=0.004, first_bucket_mb=0.002))
    m.compile([x], is_train=True, use_graph=True)
    log("compiled")
    for i in range(steps):
        log("step", i)
        _, loss = m(x, y)
        log("step done", i)
    torch.cuda.current_stream().synchronize()
    log("synced")
    return float(loss.data.float().cpu())


def main():
    from singa_amd.parallel import loop as LP

    orig_capture = LP._RankGraph.capture

    def capture(self, fn, *a, **k):
        log("capture enter")
        out = orig_capture(self, fn, *a, **k)
        log("capture exit")
        return out
    LP._RankGraph.capture = capture
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    if len(sys.argv) > 2 and sys.argv[2] == "nooverlap":
        from singa_amd.parallel import distopt
        orig = distopt.DistOpt.__init__

        def init(self, *a, **k):
            orig(self, *a, **k)
            self.overlap = False
        distopt.DistOpt.__init__ = init
    res = LP.run_ranks(rank_fn, world, 4, device=torch.device("cuda", 0), timeout_s=60.0, captured=True)
    log("results", res)


if __name__ == "__main__":
    main()
