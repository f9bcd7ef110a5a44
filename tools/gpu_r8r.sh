#!/bin/bash
# round 6, call r: bnres small GEMMs into the pre-zeroed arena, AlexNet one-pass input prep: tests + benches
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "400 t_r.log python -u -m pytest tests/test_bnres_gpu.py tests/test_models_gpu.py -k 'bnres or alexnet or tail or resnet' -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_r.log && exit 1
tools/gpu_step.sh "300 r_res1.log python bench.py --steps 20 --warmup 5" "300 r_alex1.log python bench.py --model alexnet --steps 30 --warmup 5" \
  "300 r_res2.log python bench.py --steps 20 --warmup 5" "300 r_alex2.log python bench.py --model alexnet --steps 30 --warmup 5" || exit $?
