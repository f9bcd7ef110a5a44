#!/bin/bash
# round 6, call 9h: epilogue global loads hoisted above the LDS staging: tests, act-grad microbench, benches, step kernels
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "600 t_9h.log python -u -m pytest tests/test_kernels_gpu.py tests/test_bnres_gpu.py tests/test_generic_gemm_gpu.py tests/test_stgemm_gpu.py tests/test_conv3x3_gpu.py tests/test_bert_fused_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_9h.log && exit 1
rm -rf gpurun_out/ag
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/ag -o ag --output-format rocpd -- python3 tools/bench_actgrad.py > gpurun_out/ag.log 2>&1 || exit $?
tools/gpu_step.sh "200 h_r50_1.log python bench.py --steps 20 --warmup 5" "200 h_r50_2.log python bench.py --steps 20 --warmup 5" \
  "200 h_bert_1.log python bench.py --model bert --steps 30 --warmup 5" "200 h_bert_2.log python bench.py --model bert --steps 30 --warmup 5" || exit $?
rm -rf gpurun_out/pf
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pf -o r50 --output-format rocpd -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/pf.log 2>&1 || exit $?
python3 tools/step_kernels.py $(find gpurun_out/pf -name 'r50_results.db' | head -1) > gpurun_out/r6/r50_step_kernels_r9h.txt
rm -rf gpurun_out/pf
