#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_bnres_r5t.log python -u -m pytest tests/test_bnres_gpu.py tests/test_models_gpu.py -x -q -s -k 'bnres or strided or resnet or lazy' --timeout 120 --timeout-method thread" \
  "200 bench_r5t_1.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r5t_2.log python bench.py --steps 20 --warmup 5"
