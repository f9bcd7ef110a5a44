#!/bin/bash
# fused attention backward with the bias-gradient sums: kernel time (rocprofv3) + correctness tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fa4
tools/gpu_step.sh "300 t_fa4.log python -u -m pytest tests/test_fattn_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_fa4.log && exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/fa4/d0 -o fa -- python3 tools/bench_fattn.py --iters 20 > gpurun_out/fa4/d0.log 2>&1 || exit $?
