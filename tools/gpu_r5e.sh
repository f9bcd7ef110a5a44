#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "200 bnres_test_r5e.log python -u -m pytest tests/test_bnres_gpu.py -x -v -s --timeout 120 --timeout-method thread" \
  "400 gputest_r5e.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200 bench_r5e.log python bench.py --steps 20 --warmup 5" || exit $?
bash tools/prof_step.sh r5e
