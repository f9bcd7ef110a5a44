#!/bin/bash
# One-step dispatch timeline of the AlexNet b512 training step -> gpurun_out/bert_timeline.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_bert -o bert --output-format rocpd -- python3 tools/bench_suite.py --which bert --steps 3 --warmup 2 --no-graph > gpurun_out/tl_bert.log 2>&1 || exit $?
db=$(find gpurun_out/tl_bert -name '*.db' | head -1)
python3 tools/step_timeline.py "$db" > gpurun_out/bert_timeline.txt
rm -rf gpurun_out/tl_bert
