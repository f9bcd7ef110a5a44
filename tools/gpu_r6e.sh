#!/bin/bash
# A/B of GEMM dispatch knobs on the b1024 step (alternating, same box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 ab_e_base1.log $B" \
  "200 ab_e_k6_4.log env SG_TUNE=6=4 $B" \
  "200 ab_e_k6_6.log env SG_TUNE=6=6 $B" \
  "200 ab_e_nt.log env SG_TUNE=8=1 $B" \
  "200 ab_e_base2.log $B" \
  "200 ab_e_k6_4b.log env SG_TUNE=6=4 $B" \
  "200 ab_e_k6_6b.log env SG_TUNE=6=6 $B" \
  "200 ab_e_ntb.log env SG_TUNE=8=1 $B" \
  "200 ab_e_base3.log $B"
