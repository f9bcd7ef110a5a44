#!/bin/bash
# One GPU session: every GPU test, the flagship bench, the secondary-config
# suite (BERT / sonnx-BERT graph mode, AlexNet, MLP) and the AlexNet profile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "600 gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200 bench.log python bench.py --steps 20 --warmup 5" \
  "300 suite.log python tools/bench_suite.py --which bert,bert_sonnx,alexnet,mlp_gpu --steps 20 --warmup 5" || exit $?
bash tools/alexnet_prof.sh
