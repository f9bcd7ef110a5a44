#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "200 bnres_test_r5f.log python -u -m pytest tests/test_bnres_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "200 bench_r5f.log python bench.py --steps 20 --warmup 5" || exit $?
bash tools/prof_step.sh r5f && bash tools/step_roofline.sh r5f
