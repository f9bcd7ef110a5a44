#!/bin/bash
# round 5: dynamic work queues -- GPU tests, interference rehearsal, bench, 2-rank self-launch rehearsal
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 gputest_r5b.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200 bench_r5b.log python bench.py --steps 20 --warmup 5" \
  "200 hog_kernels_r5b.log python tools/cu_hog_bench.py --what kernels --hogs 0,16,32,64" \
  "300 hog_step_r5b.log python tools/cu_hog_bench.py --what step --hogs 0,16,32 --steps 5" \
  "300 selflaunch_r5b.log env SINGA_DIST_BACKEND=gloo python bench.py --gpus 2 --batch 128 --steps 3 --warmup 1 --no-ps-parity"
