#!/bin/bash
# round 6, call 9e: GELU backward in fc2's dgrad epilogue: tests + BERT / sonnx A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "400 t_9e.log python -u -m pytest tests/test_bert_fused_gpu.py tests/test_models_gpu.py tests/test_generic_gemm_gpu.py -k 'bert or sonnx or gelu or act or mlp' -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_9e.log && exit 1
for i in 1 2; do
  tools/gpu_step.sh "200 e_on$i.log python bench.py --model bert --steps 30 --warmup 5" \
    "200 e_off$i.log env SINGA_AMD_ACT_GRAD_FUSE=0 python bench.py --model bert --steps 30 --warmup 5" || exit $?
done
tools/gpu_step.sh "400 e_sonnx.log python -u tools/bench_suite.py --which bert_sonnx --out gpurun_out/r6/bench_suite_sonnx_r9e.jsonl" || exit $?
