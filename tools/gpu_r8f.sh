#!/bin/bash
# round 6, call f: 1x1 GEMM policy map; non-chaotic ResNet-50 parity (bf16 + fp32)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "300 f_1x1.log python -u tools/bench_1x1.py --out gpurun_out/r6/bench_1x1_policies.jsonl" \
  "400 f_par_g0.log python -u tools/check_resnet_vs_torch.py --grads --batch 128 --steps 12 --gamma3 0 --modes eager --out gpurun_out/r6/resnet50_parity_gamma0_bf16.json" \
  "400 f_par_g01.log python -u tools/check_resnet_vs_torch.py --grads --batch 128 --steps 12 --gamma3 0.1 --modes eager --out gpurun_out/r6/resnet50_parity_gamma01_bf16.json" \
  "400 f_par_f32.log python -u tools/check_resnet_vs_torch.py --grads --batch 64 --steps 12 --gamma3 0.1 --dtype fp32 --modes eager --out gpurun_out/r6/resnet50_parity_gamma01_fp32.json"
