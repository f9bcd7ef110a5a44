#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_dal_r5r.log python -u -m pytest tests/test_bert_fused_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -s -k 'drop_add or bert or layernorm or linear' --timeout 120 --timeout-method thread" \
  "300 suite_r5r.log python tools/bench_suite.py --which bert,bert_sonnx --steps 20 --warmup 5" \
  "300 suite_r5r_off.log env SINGA_AMD_FUSED_DAL=0 python tools/bench_suite.py --which bert --steps 20 --warmup 5"
