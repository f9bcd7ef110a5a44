"""Which Python lines launch a training step's kernels: one eager step of a
bench.py model (after warm-up) with SG_LAUNCH_TRACE=1 (ops/native.py), every binding
call counted by (binding, call site, caller).

    SG_LAUNCH_TRACE=1 python tools/launch_sites.py [--model resnet50|alexnet|bert|bert_sonnx] [--batch 64]
"""
import argparse
import os
import sys

os.environ["SG_LAUNCH_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50", help="any bench.py --model, or bert_sonnx")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--top", type=int, default=80)
    a = ap.parse_args()
    import bench
    from singa_amd import device
    from singa_amd.ops import native as N
    from singa_amd.parallel import DistOpt

    if a.model == "bert_sonnx":  # tools/bench_suite.py's sonnx-imported BERT-base, its plain Adam
        from singa_amd import opt, sonnx, tensor
        from singa_amd.models import bert
        from singa_amd.sonnx import onnx_proto as P

        cpu = device.get_default_device()
        src = bert.bert_base(dropout=0.0, compute_dtype=torch.float32)
        ids_cpu = tensor.from_numpy(np.zeros((2, a.seq), np.int64), cpu)
        src.compile([ids_cpu], is_train=False)
        blob = sonnx.to_onnx(src, [ids_cpu]).SerializeToString()
        del src
        dev = device.create_rocm_gpu_on(0, set_default=True)
        m = sonnx.SONNXModel(P.load_model(blob), dev, compute_dtype=torch.bfloat16)
        rng = np.random.RandomState(0)
        inputs = (tensor.from_numpy(rng.randint(0, 30522, (a.batch, a.seq)).astype(np.int64), dev),
                  tensor.from_numpy(rng.randint(0, 2, a.batch).astype(np.int32), dev))
        m.set_optimizer(opt.Adam(1e-4))
    else:
        dev = device.create_rocm_gpu_on(0, set_default=True)
        args = bench._parser().parse_args(["--model", a.model, "--batch", str(a.batch), "--seq", str(a.seq)])
        m, inputs, o, _ = bench._build(args, dev, 0)
        m.set_optimizer(DistOpt(o, world_size=1, rank=0, local_rank=0))  # bench.py's fused update
    m.compile([inputs[0]], is_train=True, use_graph=False)
    m.train()
    for _ in range(2):
        m(*inputs)
    torch.cuda.synchronize()
    L = N.lib()
    L.enabled = True
    m(*inputs)
    torch.cuda.synchronize()
    L.enabled = False
    tot = sum(L.counts.values())
    byname = {}
    for (k, site), c in L.counts.items():
        byname[k] = byname.get(k, 0) + c
    print(f"# {tot} binding calls in one step")
    for k, c in sorted(byname.items(), key=lambda kv: -kv[1]):
        print(f"{c:6d}  {k}")
    print("# by call site")
    for (k, site), c in L.counts.most_common(a.top):
        print(f"{c:6d}  {k:28s} {site}")


if __name__ == "__main__":
    main()
