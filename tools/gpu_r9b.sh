#!/bin/bash
# round 6, call 9b: native tensor handle on the device pool
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_9b.log python -u -m pytest tests/test_native_tensor_gpu.py tests/test_native_tensor_cpu.py tests/test_memory_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_9b.log && exit 1
exit 0
