#!/bin/bash
# round 6, call z: idle time between kernels inside the captured ResNet-50 step (db kept)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tz -o r50 --output-format rocpd -- python3 bench.py --steps 6 --warmup 3 > gpurun_out/tz_r50.log 2>&1 || exit $?
