#!/bin/bash
# one-at-a-time sweep of the dispatch knobs on the final build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 s_base1.log $B" "200 s_k7.log env SG_TUNE=7=0 $B" "200 s_k2.log env SG_TUNE=2=0 $B" \
  "200 s_k10a.log env SG_TUNE=10=512 $B" "200 s_k10b.log env SG_TUNE=10=2048 $B" "200 s_k13.log env SG_TUNE=13=0 $B" \
  "200 s_base2.log $B" "200 s_k14.log env SG_TUNE=14=-1 $B" "200 s_k8.log env SG_TUNE=8=1 $B" "200 s_k5.log env SG_TUNE=5=0 $B" \
  "200 s_bw.log env SG_BNRES_TUNE=0=0 $B" "200 s_base3.log $B"
