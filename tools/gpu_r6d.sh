#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_stem_r6d.log python -u -m pytest tests/test_models_gpu.py -x -q -k 'pairs or paired_stem' --timeout 120 --timeout-method thread" \
  "200 bench_r6d_1.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r6d_2.log python bench.py --steps 20 --warmup 5" && tools/prof_step.sh r6d
