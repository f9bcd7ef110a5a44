#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 z_base1.log $B" "200 z_k62a.log env SG_TUNE=6=2 $B" "200 z_k60a.log env SG_TUNE=6=0 $B" \
  "200 z_base2.log $B" "200 z_k62b.log env SG_TUNE=6=2 $B" "200 z_k60b.log env SG_TUNE=6=0 $B" \
  "200 z_base3.log $B" "200 z_k62c.log env SG_TUNE=6=2 $B" "200 z_k60c.log env SG_TUNE=6=0 $B"
