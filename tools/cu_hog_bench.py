"""Interference rehearsal for the persistent kernels (verdict r4, item 1b).

At N > 1 the bucketed gradient all-reduce runs on the comm stream during the
backward, and RCCL's channel kernels occupy CUs.  A persistent kernel whose
grid is one workgroup per CU with work split STATICALLY by blockIdx then
straggles: every workgroup that cannot get a CU runs its whole share after
the others.  This tool stands a "CU hog" in for RCCL -- ``ncu`` workgroups on
a side stream, each holding (nearly) a whole CU's LDS and sleeping for the
measured span -- and times

* ``--what kernels``: each persistent kernel alone (sk_gemm_k on two 1x1-conv
  shapes, the stage-1 conv3x3_k forward, the stem forward), and
* ``--what step``: the ResNet-50 b1024 training step (bench.py's),

with the dynamic work queue on and off (``workq_set``), for hog sizes
``--hogs``.  One JSON line per measurement.

  python tools/cu_hog_bench.py --what kernels --hogs 0,16,32,64
  python tools/cu_hog_bench.py --what step --hogs 0,32 --batch 1024 --steps 6
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from singa_amd.ops import native as N  # noqa: E402


def hog(L, side, ncu, us, started=None):
    if ncu > 0:
        L.cu_hog(ncu, float(us), 0, 0 if started is None else started.data_ptr(), side.cuda_stream)


def timed(L, fn, iters, ncu, side, est_ms, started):
    """Mean ms of fn over iters launches while ncu CUs are hogged."""
    fn()
    torch.cuda.synchronize()
    started.zero_()
    hog(L, side, ncu, (est_ms * iters * 1.5 + 2.0) * 1e3, started)
    # a 50 us single-CU spin on the main stream first, so the hog's workgroups
    # are resident before the measured kernels start
    L.cu_hog(1, 50.0, 0, 0, N.stream())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters, int(started.item())


def kernels(a, L, side, started):
    dev = torch.device("cuda", 0)
    s = N.stream()
    n = a.batch
    cases = {}
    # 1x1-conv GEMMs on sk_gemm_k: stage-1 conv3 forward (64 -> 256, one K-tile)
    # and stage-2 conv3 forward (128 -> 512, two K-tiles)
    for name, (h, c, k) in {"sk_1x1_56_64x256": (56, 64, 256), "sk_1x1_28_128x512": (28, 128, 512)}.items():
        x = torch.randn(n, h, h, c, device=dev).bfloat16()
        w = (torch.randn(k, 1, 1, c, device=dev) * 0.1).bfloat16()
        y = torch.empty(n, h, h, k, device=dev, dtype=torch.bfloat16)
        ws = torch.zeros(32 * 2 * k, dtype=torch.float32, device=dev)

        def f(x=x, w=w, y=y, ws=ws, h=h, c=c, k=k):
            L.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, n, h, h, c, k, 1, 1, h, h, 1, 1, 0, 0, 1, 1, 0, 0,
                       s, ws.data_ptr())
        cases[name] = (f, (x, w, y, ws))
    x = torch.randn(n, 56, 56, 64, device=dev).bfloat16()
    w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).bfloat16()
    y = torch.empty_like(x)
    ws = torch.zeros(32 * 2 * 64, dtype=torch.float32, device=dev)

    def c3(x=x, w=w, y=y, ws=ws):
        L.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, n, 56, 56, 64, 64, 3, 3, 56, 56, 1, 1, 1, 1, 1, 1, 0, 0,
                   s, ws.data_ptr())
    cases["conv3x3_56_64"] = (c3, (x, w, y, ws))
    xp = torch.randn(n, 224, 225, 8, device=dev).bfloat16()
    wp = (torch.randn(64, 224, device=dev) * 0.05).bfloat16()
    ys = torch.empty(n, 112, 112, 64, device=dev, dtype=torch.bfloat16)
    wss = torch.zeros(32 * 2 * 64, dtype=torch.float32, device=dev)

    def stem(xp=xp, wp=wp, ys=ys, wss=wss):
        if not L.stem_fwd(xp.data_ptr(), wp.data_ptr(), ys.data_ptr(), wss.data_ptr(), n, 224, 225, 112, 112, s):
            raise RuntimeError("stem kernel did not take the shape")
    cases["stem_224"] = (stem, (xp, wp, ys, wss))
    for name, (fn, bufs) in cases.items():
        # outputs of both paths agree (the queue only reorders the work)
        outs = {}
        for q in (1, 0):
            L.workq_set(q)
            fn()
            torch.cuda.synchronize()
            outs[q] = [bufs[2].clone()]
        same = all(torch.equal(a_, b_) for a_, b_ in zip(outs[0], outs[1]))
        base = None
        for k in a.hogs:
            for q in (1, 0):
                L.workq_set(q)
                ms, got = timed(L, fn, a.iters, k, side, (base or 2.0), started)
                if k == 0 and q == 1:
                    base = ms
                print(json.dumps({"kernel": name, "hog_cus": k, "hog_resident": got, "queue": bool(q),
                                  "ms": round(ms, 4), "vs_unhogged_queue": round(ms / base, 3) if base else None,
                                  "ideal": round(L.cu_count() / max(1, L.cu_count() - k), 3),
                                  "outputs_equal_queue_vs_static": same}), flush=True)
    L.workq_set(1)


def step(a, L, side, started):
    from singa_amd import device, opt, tensor
    from singa_amd.models import resnet
    from singa_amd.parallel import DistOpt, init_distributed
    import numpy as np

    dev = device.create_rocm_gpu_on(0, set_default=True)
    dev.SetRandSeed(1234)
    comm = init_distributed(rank=0, world_size=1, local_rank=0)
    m = resnet.create_model(50, num_classes=1000, compute_dtype=torch.bfloat16)
    m.set_optimizer(DistOpt(opt.SGD(lr=0.01, momentum=0.9, weight_decay=1e-4), comm=comm))
    B = a.batch
    rng = np.random.RandomState(0)
    tx = tensor.from_numpy(rng.standard_normal((B, 3, 224, 224)).astype(np.float32), dev)
    ty = tensor.from_numpy(rng.randint(0, 1000, size=(B,)).astype(np.int32), dev)
    m.compile([tx], is_train=True, use_graph=False)
    m.train()
    for _ in range(3):
        m(tx, ty)
    torch.cuda.synchronize()
    base = None
    for k in a.hogs:
        for q in (1, 0):
            L.workq_set(q)
            m(tx, ty)
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.steps):
                started.zero_()
                torch.cuda.synchronize()
                # the hog covers the whole (possibly slowed) step; the step is
                # timed with events on its own stream, not to the host sync
                # (which also waits for the hog to run out)
                hog(L, side, k, (base or 80.0) * 2.5e3, started)
                L.cu_hog(1, 50.0, 0, 0, N.stream())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                m(tx, ty)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = sorted(ts)[len(ts) // 2]
            if k == 0 and q == 1:
                base = ms
            print(json.dumps({"what": "resnet50_step", "batch": B, "hog_cus": k, "hog_resident": int(started.item()),
                              "queue": bool(q), "ms_median": round(ms, 2), "ms_all": [round(t, 2) for t in ts],
                              "vs_unhogged_queue": round(ms / base, 3) if base else None,
                              "ideal": round(L.cu_count() / max(1, L.cu_count() - k), 3)}), flush=True)
    L.workq_set(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=("kernels", "step"), default="kernels")
    ap.add_argument("--hogs", default="0,16,32,64")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    a.hogs = [int(v) for v in a.hogs.split(",")]
    L = N.lib()
    side = torch.cuda.Stream()
    started = torch.zeros(1, dtype=torch.int32, device="cuda")
    print(json.dumps({"cu_count": L.cu_count()}), flush=True)
    (kernels if a.what == "kernels" else step)(a, L, side, started)


if __name__ == "__main__":
    main()
