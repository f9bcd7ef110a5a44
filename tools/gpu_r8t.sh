#!/bin/bash
# round 6, call t: Linear data gradients accumulate into the pending residual gradient: tests + BERT A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "400 t_t.log python -u -m pytest tests/test_bert_fused_gpu.py tests/test_models_gpu.py -k 'bert or sonnx or mlp or alexnet' -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_t.log && exit 1
tools/gpu_step.sh "300 t_on1.log python bench.py --model bert --steps 30 --warmup 5" \
  "300 t_off1.log env SINGA_AMD_INPLACE_ACC=0 python bench.py --model bert --steps 30 --warmup 5" \
  "300 t_on2.log python bench.py --model bert --steps 30 --warmup 5" \
  "300 t_off2.log env SINGA_AMD_INPLACE_ACC=0 python bench.py --model bert --steps 30 --warmup 5" \
  "400 t_sonnx.log python -u tools/bench_suite.py --which bert_sonnx --out gpurun_out/r6/bench_suite_sonnx_r8t.jsonl" || exit $?
