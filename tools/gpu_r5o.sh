#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_ln_r5o.log python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'layernorm or unary or softmax' --timeout 120 --timeout-method thread" \
  "200 elem_r5o2.log python tools/bert_elem_bench.py" \
  "300 suite_r5o.log python tools/bench_suite.py --which bert,bert_sonnx --steps 20 --warmup 5"
