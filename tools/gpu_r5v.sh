#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "200 bench_r5v_lazy1.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r5v_place1.log env SINGA_AMD_STRIDED_LAZY=0 python bench.py --steps 20 --warmup 5" \
  "200 bench_r5v_lazy2.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r5v_place2.log env SINGA_AMD_STRIDED_LAZY=0 python bench.py --steps 20 --warmup 5"
