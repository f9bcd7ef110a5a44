#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 t_r6p.log python -u -m pytest tests/test_kernels_gpu.py -q -k 'wgrad_256x128 or big or conv_fwd_bwd' --timeout 120 --timeout-method thread -p no:cacheprovider" && \
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 w_off1.log $B" "200 w_on1.log env SG_TUNE=15=1 $B" "200 w_off2.log $B" "200 w_on2.log env SG_TUNE=15=1 $B" "200 w_off3.log $B" "200 w_on3.log env SG_TUNE=15=1 $B" && \
tools/gpu_step.sh "200 wsweep_on.log env SG_TUNE=15=1 python tools/wgrad_sweep.py" "200 wsweep_off.log python tools/wgrad_sweep.py"
