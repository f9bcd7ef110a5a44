#!/bin/bash
# round 6, call 9a: gated exact BN reduction on a small grid: tests, ResNet-50 bench x2, step kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "500 t_9a.log python -u -m pytest tests/test_models_gpu.py tests/test_bnres_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_9a.log && exit 1
tools/gpu_step.sh "200 a_r50_1.log python bench.py --steps 20 --warmup 5" "200 a_r50_2.log python bench.py --steps 20 --warmup 5" || exit $?
rm -rf gpurun_out/tz
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tz -o r50 --output-format rocpd -- python3 bench.py --steps 6 --warmup 3 > gpurun_out/tz_r50.log 2>&1 || exit $?
