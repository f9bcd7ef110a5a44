#!/bin/bash
# round 6, call h: restricted streaming GEMM (default on) A/B; fp32 parity in the zero-gamma regime
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "300 t_st.log python -u -m pytest tests/test_stgemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_st.log && exit 1
tools/gpu_step.sh "200 h_on1.log $B" "200 h_off1.log SG_TUNE=18=0 $B" "200 h_on2.log $B" "200 h_off2.log SG_TUNE=18=0 $B" "200 h_on3.log $B" "200 h_off3.log SG_TUNE=18=0 $B" \
  "400 h_par_f32g0.log python -u tools/check_resnet_vs_torch.py --grads --batch 64 --steps 12 --gamma3 0 --dtype fp32 --modes eager --out gpurun_out/r6/resnet50_parity_gamma0_fp32.json" \
  "400 h_par_f32det.log SINGA_AMD_DETERMINISTIC=1 python -u tools/check_resnet_vs_torch.py --grads --batch 64 --steps 12 --gamma3 0.1 --dtype fp32 --modes eager --out gpurun_out/r6/resnet50_parity_gamma01_fp32_det.json"
