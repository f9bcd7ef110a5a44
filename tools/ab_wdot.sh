#!/bin/bash
# Identity-sum BN backward: its GPU tests, then an A/B of the flagship bench
# (SINGA_AMD_BN_WDOT=0/1, alternating) and a kernel profile with it on.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tools/gpu_step.sh "300 gt_wdot.log python -u -m pytest tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'identity_sum or stacked_bottlenecks or resnet'" || exit 1
grep -q " passed" gpurun_out/gt_wdot.log && ! grep -q "failed" gpurun_out/gt_wdot.log || exit 1
for i in 1 2; do for v in 0 1; do SINGA_AMD_BN_WDOT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ps-parity > gpurun_out/ab_tmp.log 2>&1 || { tail -20 gpurun_out/ab_tmp.log; exit 1; }; echo "$i wdot=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_tmp.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/ab_tmp.log)" | tee -a gpurun_out/ab_wdot.txt; done; done
SINGA_AMD_BN_WDOT=1 bash tools/prof_step.sh wdot2
