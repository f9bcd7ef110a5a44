#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "600 t_r6o.log python -u -m pytest tests/test_kernels_gpu.py tests/test_bert_fused_gpu.py tests/test_models_gpu.py tests/test_generic_gemm_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider" && \
tools/gpu_step.sh "300 s_r6o.log python tools/bench_suite.py --which bert,bert_sonnx,alexnet,mlp_gpu --out gpurun_out/bench_suite_r6o.jsonl" \
  "200 r_r6o_1.log python bench.py --steps 20 --warmup 5" "200 r_r6o_2.log python bench.py --steps 20 --warmup 5"
