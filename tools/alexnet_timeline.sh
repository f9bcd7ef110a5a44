#!/bin/bash
# One-step dispatch timeline of the AlexNet b512 training step -> gpurun_out/alexnet_timeline.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_alex -o alex --output-format rocpd -- python3 tools/bench_suite.py --which alexnet --steps 3 --warmup 2 --no-graph > gpurun_out/tl_alex.log 2>&1 || exit $?
db=$(find gpurun_out/tl_alex -name '*.db' | head -1)
python3 tools/step_timeline.py "$db" > gpurun_out/alexnet_timeline.txt
rm -rf gpurun_out/tl_alex
