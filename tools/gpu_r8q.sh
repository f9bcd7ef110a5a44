#!/bin/bash
# round 6, call q: dgrad / wgrad concurrency probe on the ResNet-50 b1024 conv shapes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "300 q_overlap.log python -u tools/probe_overlap.py --iters 10 --out gpurun_out/r6/probe_overlap.jsonl" || exit $?
