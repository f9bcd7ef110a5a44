#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 t_r6s_a.log env SG_TUNE=16=3 SG_BNRES_TUNE=1=1 python -u -m pytest tests/test_kernels_gpu.py tests/test_bnres_gpu.py -q -k 'conv or bnres or gsum or tail' --timeout 120 --timeout-method thread -p no:cacheprovider" && \
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 x_base1.log $B" "200 x_k1a.log env SG_TUNE=16=1 $B" "200 x_k2a.log env SG_TUNE=16=2 $B" "200 x_bd1.log env SG_BNRES_TUNE=1=1 $B" \
  "200 x_base2.log $B" "200 x_k1b.log env SG_TUNE=16=1 $B" "200 x_k2b.log env SG_TUNE=16=2 $B" "200 x_bd2.log env SG_BNRES_TUNE=1=1 $B" \
  "200 x_base3.log $B" "200 x_k3a.log env SG_TUNE=16=3 $B"
