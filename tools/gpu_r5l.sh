#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "600 parity_r5l.log python -u tools/check_resnet_vs_torch.py --grads --batch 128 --steps 12 --lr 0.02 --modes eager"
