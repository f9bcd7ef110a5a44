#!/bin/bash
# Rehearse the N>1 bench path on ONE GPU: 2 ranks over gloo (GPU tensors are
# staged through the host), small batch so both replicas fit.
cd "$GRAFT_REPO_ROOT"
export SINGA_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --batch ${1:-128} --steps ${2:-5} --warmup ${3:-2}
