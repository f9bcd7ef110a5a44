#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "600 t_r6x.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider" && \
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 u_new1.log $B" "200 u_k61a.log env SG_TUNE=6=1 $B" "200 u_k68a.log env SG_TUNE=6=8 $B" \
  "200 u_new2.log $B" "200 u_k61b.log env SG_TUNE=6=1 $B" "200 u_k68b.log env SG_TUNE=6=8 $B" \
  "200 u_mlp.log python tools/bench_suite.py --which mlp_gpu"
