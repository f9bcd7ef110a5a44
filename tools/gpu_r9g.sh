#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/ag
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/ag -o ag --output-format rocpd -- python3 tools/bench_actgrad.py > gpurun_out/ag.log 2>&1 || exit $?
