#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 t_r6r.log python -u -m pytest tests/test_bnres_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider" && \
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 v_new1.log $B" "200 v_old1.log env SG_BNRES_TUNE=0=0 $B" "200 v_new2.log $B" "200 v_old2.log env SG_BNRES_TUNE=0=0 $B" "200 v_new3.log $B" "200 v_old3.log env SG_BNRES_TUNE=0=0 $B"
