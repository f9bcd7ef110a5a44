#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 t_r6t.log python -u -m pytest tests/test_kernels_gpu.py -q -k 'wgrad_256x128 or persistent_short_k' --timeout 120 --timeout-method thread -p no:cacheprovider" && \
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 y_base1.log $B" "200 y_k17a.log env SG_TUNE=17=1 $B" "200 y_base2.log $B" "200 y_k17b.log env SG_TUNE=17=1 $B" "200 y_base3.log $B" "200 y_k17c.log env SG_TUNE=17=1 $B" && \
tools/gpu_step.sh "200 ysweep_on.log env SG_TUNE=17=1 python tools/wgrad_sweep.py" "200 ysweep_off.log python tools/wgrad_sweep.py"
