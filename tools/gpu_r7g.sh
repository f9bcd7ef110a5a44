#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 sl4_graph.log env SINGA_DIST_BACKEND=gloo python bench.py --gpus 4 --batch 64 --steps 3 --warmup 2 --no-ps-parity" \
  "400 sl4_eager.log env SINGA_DIST_BACKEND=gloo python bench.py --gpus 4 --batch 64 --steps 3 --warmup 2 --no-ps-parity --eager"
