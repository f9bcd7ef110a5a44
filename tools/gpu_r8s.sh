#!/bin/bash
# round 6, call s: fc1 bias gradient in fc2's dgrad epilogue (gemm_act stats mode 5): tests + BERT benches
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "400 t_s.log python -u -m pytest tests/test_generic_gemm_gpu.py tests/test_bert_fused_gpu.py tests/test_fattn_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_s.log && exit 1
tools/gpu_step.sh "300 s_on1.log python bench.py --model bert --steps 30 --warmup 5" \
  "300 s_off1.log env SINGA_AMD_BIAS_INPLACE=0 python bench.py --model bert --steps 30 --warmup 5" \
  "300 s_on2.log python bench.py --model bert --steps 30 --warmup 5" \
  "400 s_sonnx.log python -u tools/bench_suite.py --which bert_sonnx --out gpurun_out/r6/bench_suite_sonnx_r8s.jsonl" || exit $?
