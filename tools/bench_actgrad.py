"""fc2's data-gradient GEMM at BERT-base shapes (dy [4096, 768] x W2 [3072,
768]^T -> [4096, 3072]): plain, with the GELU derivative in the epilogue, and
with the producer's bias-gradient column sums too; rocprofv3 gives the kernel
times (each variant runs --iters times in a row)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from singa_amd.ops import functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    dy = torch.randn(4096, 768, device="cuda", generator=g).bfloat16()
    w = (torch.randn(3072, 768, device="cuda", generator=g) * 0.05).bfloat16()
    z = torch.randn(4096, 3072, device="cuda", generator=g).bfloat16()
    cs = torch.zeros(3072, device="cuda")
    acc = torch.zeros(4096, 3072, device="cuda").bfloat16()
    for name, fn in [("plain", lambda: F.gemm_nt(dy, w, out_dtype=torch.bfloat16)),
                     ("act", lambda: F.gemm_nt(dy, w, out_dtype=torch.bfloat16, act_grad=("gelu", z))),
                     ("act_cs", lambda: F.gemm_nt(dy, w, out_dtype=torch.bfloat16, act_grad=("gelu", z), colsum_c=cs)),
                     ("act_relu", lambda: F.gemm_nt(dy, w, out_dtype=torch.bfloat16, act_grad=("relu", z))),
                     ("act_tanh", lambda: F.gemm_nt(dy, w, out_dtype=torch.bfloat16, act_grad=("tanh", z))),
                     ("beta1", lambda: F.gemm(dy, w, tb=True, out=acc, beta=1.0))]:
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        print(name, flush=True)


if __name__ == "__main__":
    main()
