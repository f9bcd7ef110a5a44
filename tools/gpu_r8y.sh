#!/bin/bash
# round 6, call y: LDS-only barriers in the staged GEMM epilogue (knob 19): GEMM / conv tests + ResNet-50 / AlexNet / BERT A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "500 t_y.log python -u -m pytest tests/test_kernels_gpu.py tests/test_bnres_gpu.py tests/test_stgemm_gpu.py tests/test_generic_gemm_gpu.py tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_y.log && exit 1
for i in 1 2; do
  tools/gpu_step.sh "200 y_new$i.log python bench.py --steps 20 --warmup 5" "200 y_old$i.log env SG_TUNE=19=1 python bench.py --steps 20 --warmup 5" || exit $?
done
tools/gpu_step.sh "200 y_anew.log python bench.py --model alexnet --steps 30 --warmup 5" "200 y_aold.log env SG_TUNE=19=1 python bench.py --model alexnet --steps 30 --warmup 5" \
  "200 y_bnew.log python bench.py --model bert --steps 30 --warmup 5" "200 y_bold.log env SG_TUNE=19=1 python bench.py --model bert --steps 30 --warmup 5" || exit $?
