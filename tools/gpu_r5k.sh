#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 bnres_r5k.log python -u -m pytest tests/test_bnres_gpu.py tests/test_workq_gpu.py -x -v -s --timeout 120 --timeout-method thread" \
  "200 bench_r5k_on.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r5k_off.log env SINGA_AMD_TAIL_RECOMPUTE=0 python bench.py --steps 20 --warmup 5" \
  "200 bench_r5k_on2.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r5k_off2.log env SINGA_AMD_TAIL_RECOMPUTE=0 python bench.py --steps 20 --warmup 5"
