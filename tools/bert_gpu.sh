#!/bin/bash
# GPU session for the BERT path: kernel numerics + BERT model tests, the
# BERT / sonnx-BERT suite in graph and eager mode, and a kernel profile of the
# native BERT-base step (summary -> gpurun_out/prof_bert.txt).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "600 t_bert.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" "300 suite_graph.log python tools/bench_suite.py --which bert,bert_sonnx --steps 20 --warmup 5" "300 suite_eager.log python tools/bench_suite.py --which bert,bert_sonnx --steps 20 --warmup 5 --no-graph" "300 prof_bert.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o bert --output-format rocpd -- python3 tools/bench_suite.py --which bert --steps 10 --warmup 3 --no-graph" || exit $?
db=$(find gpurun_out/prof_bert -name '*.db' | head -1)
python3 tools/prof_summary.py "$db" --steps 13 > gpurun_out/prof_bert.txt
rm -rf gpurun_out/prof_bert
