#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 bnres_r5m.log python -u -m pytest tests/test_bnres_gpu.py -x -v -s --timeout 120 --timeout-method thread" \
  "200 bench_r5m_on.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r5m_off.log env SINGA_FUSED_DOWN_TAIL=0 python bench.py --steps 20 --warmup 5" \
  "200 bench_r5m_on2.log python bench.py --steps 20 --warmup 5"
