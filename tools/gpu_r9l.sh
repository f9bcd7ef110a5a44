#!/bin/bash
# round 6, call 9l: non-inlined activation helpers in the staged epilogue: tests, act-grad microbench, BERT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 t_9l.log python -u -m pytest tests/test_generic_gemm_gpu.py tests/test_bert_fused_gpu.py tests/test_models_gpu.py -k 'act or gelu or bert or mlp or sonnx' -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_9l.log && exit 1
rm -rf gpurun_out/ag
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/ag -o ag --output-format rocpd -- python3 tools/bench_actgrad.py > gpurun_out/ag.log 2>&1 || exit $?
tools/gpu_step.sh "200 l_bert1.log python bench.py --model bert --steps 30 --warmup 5" "200 l_bert2.log python bench.py --model bert --steps 30 --warmup 5" \
  "200 l_gelu1.log env SINGA_AMD_FUSE_GELU=1 python bench.py --model bert --steps 30 --warmup 5" || exit $?
