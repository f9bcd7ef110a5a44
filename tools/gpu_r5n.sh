#!/bin/bash
# BERT / sonnx-BERT suite + a kernel profile of the native BERT-base step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 suite_r5n.log python tools/bench_suite.py --which bert,bert_sonnx,mlp_gpu --steps 20 --warmup 5" \
  "300 prof_bert_r5n.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o bert --output-format rocpd -- python3 tools/bench_suite.py --which bert --steps 10 --warmup 3 --no-graph" || exit $?
db=$(find gpurun_out/prof_bert -name '*.db' | head -1)
python3 tools/prof_summary.py "$db" --steps 13 > gpurun_out/prof_bert_r5n.txt
rm -rf gpurun_out/prof_bert
