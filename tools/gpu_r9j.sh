#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
rm -rf gpurun_out/pf
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pf -o r50 --output-format rocpd -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/pf.log 2>&1 || exit $?
python3 tools/step_kernels.py $(find gpurun_out/pf -name 'r50_results.db' | head -1) > gpurun_out/r6/r50_step_kernels_r9j.txt
rm -rf gpurun_out/pf
