#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "200 bench_r6c_q1.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r6c_p1.log env SG_TUNE=13=0 python bench.py --steps 20 --warmup 5" \
  "200 bench_r6c_q2.log python bench.py --steps 20 --warmup 5" \
  "200 bench_r6c_p2.log env SG_TUNE=13=0 python bench.py --steps 20 --warmup 5" \
  "300 t_conv_r6c.log python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'wgrad or conv' --timeout 120 --timeout-method thread"
