#!/bin/bash
# round-5 baseline: bench + kernel stats of the round-4 final build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "200 bench_r5a.log python bench.py --steps 20 --warmup 5" || exit $?
bash tools/prof_step.sh r5a
