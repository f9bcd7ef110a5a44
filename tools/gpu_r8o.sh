#!/bin/bash
# round 6, call o: launch sites of one eager sonnx-imported BERT-base step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "400 ls_sonnx.log python -u tools/launch_sites.py --model bert_sonnx --batch 32 --top 150" || exit $?
cp gpurun_out/ls_sonnx.log gpurun_out/r6/launch_sites_bert_sonnx.txt
