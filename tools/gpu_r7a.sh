#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 sl_graph.log env SINGA_DIST_BACKEND=gloo python bench.py --gpus 2 --batch 128 --steps 3 --warmup 1 --no-ps-parity --graph" \
  "300 sl_eager.log env SINGA_DIST_BACKEND=gloo python bench.py --gpus 2 --batch 128 --steps 3 --warmup 1 --no-ps-parity"
