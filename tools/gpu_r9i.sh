#!/bin/bash
# round 6, call 9i: the rebuilt tree (epilogue hoist reverted): quick tests + ResNet-50 / BERT benches
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 t_9i.log python -u -m pytest tests/test_kernels_gpu.py tests/test_bnres_gpu.py tests/test_generic_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_9i.log && exit 1
tools/gpu_step.sh "200 i_r50_1.log python bench.py" "200 i_r50_2.log python bench.py" "200 i_bert.log python bench.py --model bert --steps 30 --warmup 5" || exit $?
