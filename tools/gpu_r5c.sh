#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "200 workq_check_r5c.log python tools/workq_check.py 1024" \
  "300 gputest_workq_r5c.log python -u -m pytest tests/test_workq_gpu.py tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "200 hog_kernels_r5c.log python tools/cu_hog_bench.py --what kernels --hogs 0,32" \
  "200 bench_r5c.log python bench.py --steps 20 --warmup 5" \
  "300 hog_step_r5c.log python tools/cu_hog_bench.py --what step --hogs 0,32 --steps 5"
