"""List the PyTorch calls that compute or copy device data during a workload's
training steps (the Python-side companion of tools/kernel_purity.py: purity
says WHICH torch kernels ran, this says WHERE they were called from).

Runs the bench_suite / bench.py workloads for a couple of steps under a
``TorchFunctionMode`` that records every torch call touching a CUDA tensor
other than metadata and free views, with its call site.  Allocations are
reported in their own section: every device tensor of a step should come
from the framework's native pool (singa_amd/memory.py), so a
``torch.empty``-family call producing a CUDA tensor is listed as a PyTorch
allocation, and ``torch.cuda.Stream`` / ``Event`` / ``CUDAGraph``
constructions are counted too (the framework owns its streams, events and
graphs: singa_amd/stream.py).

    python tools/torch_calls.py --which resnet50,alexnet,bert,bert_sonnx,mlp_gpu,conv_conf
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.overrides import TorchFunctionMode  # noqa: E402

ALLOW = {"__get__", "dim", "size", "stride", "numel", "data_ptr", "element_size", "is_contiguous", "view",
         "as_strided", "permute", "transpose", "t", "unsqueeze", "squeeze", "expand", "movedim", "narrow",
         "__getitem__", "numpy", "detach", "requires_grad_", "_set_grad_enabled", "storage_offset", "untyped_storage", "__len__", "__hash__", "__eq__", "is_floating_point",
         "unbind", "split", "chunk", "from_numpy", "__format__", "__repr__", "tolist", "item", "__float__", "__int__",
         "__bool__", "__index__", "view_as", "get_device", "is_complex", "has_names", "__array__", "_is_view",
         "is_pinned", "__iter__", "ndimension", "nelement", "record_stream", "cuda_stream"}
MAYBE_VIEW = {"reshape", "contiguous", "float", "to", "flatten", "long", "bfloat16"}
ALLOC = {"empty", "empty_like", "empty_strided", "zeros", "zeros_like", "ones", "ones_like", "full", "full_like",
         "rand", "randn", "arange", "tensor"}


def _cuda(x) -> bool:
    if isinstance(x, torch.Tensor):
        return x.is_cuda
    if isinstance(x, (list, tuple)):
        return any(_cuda(y) for y in x)
    return False


class Tracer(TorchFunctionMode):
    def __init__(self):
        super().__init__()
        self.calls = collections.Counter()
        self.allocs = collections.Counter()

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        r = func(*args, **kwargs)
        name = getattr(func, "__name__", str(func))
        if name in ALLOW or not (_cuda(args) or _cuda(list(kwargs.values())) or _cuda(r)):
            return r
        if (name in MAYBE_VIEW and args and isinstance(args[0], torch.Tensor) and isinstance(r, torch.Tensor)
                and r.untyped_storage().data_ptr() == args[0].untyped_storage().data_ptr()):
            return r
        site = " <- ".join(f"{f.filename.replace(os.getcwd() + '/', '')}:{f.lineno}"
                           for f in traceback.extract_stack()[-6:-1]
                           if "torch_calls.py" not in f.filename)
        if name in ALLOC:
            self.allocs[(name, site)] += 1
            return r
        self.calls[(name, site)] += 1
        return r


_CUDA_OBJS = collections.Counter()


def _count_cuda_objects():
    """Count torch.cuda.Stream / Event / CUDAGraph constructions."""
    def make(nm, orig):
        class Sub(orig):  # counting subclass
            def __new__(cls, *a, **k):
                # (an ExternalStream is the carrier of a framework-owned stream
                # handle -- singa_amd.stream.Stream -- not a PyTorch stream)
                if not issubclass(cls, getattr(torch.cuda, "ExternalStream", ())):
                    site = " <- ".join(f"{f.filename.replace(os.getcwd() + '/', '')}:{f.lineno}"
                                       for f in traceback.extract_stack()[-5:-1])
                    _CUDA_OBJS[(f"torch.cuda.{nm}", site)] += 1
                return orig.__new__(cls, *a, **k)
        Sub.__name__ = nm
        return Sub
    for nm in ("Stream", "Event", "CUDAGraph"):
        setattr(torch.cuda, nm, make(nm, getattr(torch.cuda, nm)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="resnet50,alexnet,bert,bert_sonnx,mlp_gpu,conv_conf")
    ap.add_argument("--native", default="copy_nd,fill,reduce,zero,binary_nd",
                    help="also record the call sites of these native (_C) launches")
    a = ap.parse_args()
    _count_cuda_objects()
    from singa_amd.ops import native as NN
    L = NN.lib()
    nat = collections.Counter()
    for fname in [f for f in a.native.split(",") if f and hasattr(L, f)]:
        def wrap(orig, fname=fname):
            def f(*args, **kw):
                site = " <- ".join(f"{fr.filename.replace(os.getcwd() + '/', '')}:{fr.lineno}"
                                   for fr in traceback.extract_stack()[-6:-1])
                nat[(fname, site)] += 1
                return orig(*args, **kw)
            return f
        setattr(L, fname, wrap(getattr(L, fname)))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    import bench_suite as BS

    class A:
        batch = None
        steps = 2
        warmup = 1
        no_graph = False
        seq = 128
        out = None

    for w in a.which.split(","):
        tr = Tracer()
        with tr:
            if w == "resnet50":
                # bench.py is its own process: trace it through this tool's
                # import of its main() instead
                sys.argv = ["bench.py", "--steps", "2", "--warmup", "1", "--batch", "64", "--no-ps-parity"]
                import bench
                bench.main()
            elif w == "conv_conf" or w == "mlp_conf":
                from singa_amd import main as M
                M.main(["--model_conf", f"examples/mnist/{w.split('_')[0]}.conf", "--device", "gpu", "--synthetic",
                        "--train_steps", "3"])
            else:
                fn = {"alexnet": BS.bench_alexnet, "bert": BS.bench_bert, "bert_sonnx": BS.bench_bert_sonnx,
                      "mlp_gpu": lambda x: BS.bench_mlp(x, True)}[w]
                fn(A)
        print(f"== {w}: {sum(tr.calls.values())} torch calls on device data")
        for (name, site), n in tr.calls.most_common(40):
            print(f"  {n:5d}  {name:24s} {site}")
        print(f"-- {w}: {sum(tr.allocs.values())} PyTorch allocations of device tensors")
        for (name, site), n in tr.allocs.most_common(25):
            print(f"  {n:5d}  {name:24s} {site}")
        print(f"-- {w}: {sum(_CUDA_OBJS.values())} torch.cuda Stream/Event/CUDAGraph objects")
        for (name, site), n in _CUDA_OBJS.most_common(15):
            print(f"  {n:5d}  {name:24s} {site}")
        _CUDA_OBJS.clear()
        from singa_amd import memory as MEM
        if torch.cuda.is_available():
            st = MEM.stats(torch.device("cuda", 0))
            print(f"-- {w}: native pool: peak {st.get('peak_in_use_bytes', 0) / 2**30:.2f} GiB in use, "
                  f"{st.get('reserved_bytes', 0) / 2**30:.2f} GiB reserved, {st.get('allocs', 0)} allocations, "
                  f"{st.get('cache_hits', 0)} cache hits; torch allocator: "
                  f"{torch.cuda.max_memory_allocated() / 2**30:.2f} GiB peak")
        print(f"-- {w}: native glue launches by call site")
        for (name, site), n in nat.most_common(25):
            print(f"  {n:5d}  {name:24s} {site}")
        nat.clear()
        sys.stdout.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
