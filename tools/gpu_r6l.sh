#!/bin/bash
# full GPU suite, then a kernel profile of the native BERT-base step (graph off)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "1100 gputests_r6l.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider" && \
tools/gpu_step.sh "300 prof_bert_r6l.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o bert --output-format rocpd -- python3 tools/bench_suite.py --which bert --steps 10 --warmup 3 --no-graph" || exit $?
db=$(find gpurun_out/prof_bert -name '*.db' | head -1)
python3 tools/prof_summary.py "$db" --steps 13 > gpurun_out/prof_bert_r6l.txt
python3 tools/kernel_dispatches.py "$db" "igemm_k" --steps 13 > gpurun_out/bert_dispatch_r6l.txt
rm -rf gpurun_out/prof_bert
