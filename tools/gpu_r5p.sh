#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_ln_r5p.log python -u -m pytest tests/test_kernels_gpu.py tests/test_bnres_gpu.py -x -q -k 'layernorm or unary or softmax or xent or bnres or sqnorm or clip' --timeout 120 --timeout-method thread" \
  "200 elem_r5p.log python tools/bert_elem_bench.py" \
  "300 suite_r5p.log python tools/bench_suite.py --which bert,bert_sonnx --steps 20 --warmup 5"
