#!/bin/bash
# round 6, call m: launch sites of one eager BERT / ResNet-50 step (small-kernel inventory)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "300 ls_bert.log python -u tools/launch_sites.py --model bert --batch 32 --top 120" \
  "300 ls_resnet.log python -u tools/launch_sites.py --model resnet50 --batch 64 --top 150" || exit $?
cp gpurun_out/ls_bert.log gpurun_out/r6/launch_sites_bert.txt
cp gpurun_out/ls_resnet.log gpurun_out/r6/launch_sites_resnet50.txt
