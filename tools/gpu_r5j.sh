#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 workq_r5j.log python -u -m pytest tests/test_workq_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "700 gpu_tests_r5j.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200 bench_r5j_1.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r5j_2.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r5j_3.log python bench.py --steps 20 --warmup 5"
