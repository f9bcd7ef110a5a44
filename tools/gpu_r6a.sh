#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_bnres_r6a.log python -u -m pytest tests/test_bnres_gpu.py tests/test_workq_gpu.py -q -s --timeout 120 --timeout-method thread" \
  "200 bench_r6a_on1.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r6a_on2.log python bench.py --steps 20 --warmup 5"
