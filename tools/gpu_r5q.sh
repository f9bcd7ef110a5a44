#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 t_gemm_r5q.log python -u -m pytest tests/test_generic_gemm_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k 'gemm or bert or linear or mlp' --timeout 120 --timeout-method thread" \
  "300 suite_r5q.log python tools/bench_suite.py --which bert,bert_sonnx,alexnet --steps 20 --warmup 5"
