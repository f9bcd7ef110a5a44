#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_bnres_r5z.log python -u -m pytest tests/test_bnres_gpu.py -q -s --timeout 120 --timeout-method thread" \
  "200 bench_r5z_on1.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r5z_off1.log env SINGA_AMD_GRAM_STATS=0 python bench.py --steps 20 --warmup 5" \
  "200 bench_r5z_on2.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r5z_off2.log env SINGA_AMD_GRAM_STATS=0 python bench.py --steps 20 --warmup 5"
