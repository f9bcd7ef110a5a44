#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
S="python tools/bench_suite.py --which alexnet"
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "300 t_r7e.log python -u -m pytest tests/test_kernels_gpu.py -q -k 'wgrad_256x128' --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "200 e_on1.log $S" "200 e_off1.log env SG_TUNE=15=0 $S" "200 e_on2.log $S" "200 e_off2.log env SG_TUNE=15=0 $S" \
  "200 e_r1.log $B" "200 e_r0.log env SG_TUNE=15=0 $B" "200 e_r1b.log $B" "200 e_r0b.log env SG_TUNE=15=0 $B"
