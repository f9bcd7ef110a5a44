#!/bin/bash
# final-build evidence: kernel stats + purity, two bench runs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "200 fin_b1.log python bench.py" "200 fin_b2.log python bench.py --steps 20 --warmup 5" && bash tools/prof_step.sh r6u
