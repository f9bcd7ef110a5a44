#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 t_r6q.log python -u -m pytest tests/test_kernels_gpu.py tests/test_bnres_gpu.py -q -k 'wgrad or conv or big' --timeout 120 --timeout-method thread -p no:cacheprovider" && \
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 q_new1.log $B" "200 q_old1.log env SG_TUNE=15=0 $B" "200 q_new2.log $B" "200 q_old2.log env SG_TUNE=15=0 $B" "200 q_new3.log $B" "200 q_old3.log env SG_TUNE=15=0 $B" && \
tools/gpu_step.sh "200 qsweep.log python tools/wgrad_sweep.py"
