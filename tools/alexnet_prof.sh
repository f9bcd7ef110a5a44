#!/bin/bash
# Kernel profile of the AlexNet bench_suite step (summary -> gpurun_out/prof_alexnet.txt).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_alex -o alex --output-format rocpd -- python3 tools/bench_suite.py --which alexnet --steps 10 --warmup 3 --no-graph > gpurun_out/prof_alex.log 2>&1 || exit $?
db=$(find gpurun_out/prof_alex -name '*.db' | head -1)
python3 tools/prof_summary.py "$db" --steps 13 > gpurun_out/prof_alexnet.txt
rm -rf gpurun_out/prof_alex
timeout -k 10 300 python3 tools/bench_suite.py --which alexnet,mlp_gpu --steps 20 --warmup 5 > gpurun_out/suite_alex.log 2>&1
