#!/bin/bash
# round 6, call n: bias gradients summed by their consumers (DropAddLayerNorm, fused attention): tests + BERT A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "300 t_bias.log python -u -m pytest tests/test_fattn_gpu.py tests/test_bert_fused_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_bias.log && exit 1
for i in 1 2; do
  tools/gpu_step.sh "300 n_on$i.log python bench.py --model bert --steps 30 --warmup 5" \
    "300 n_off$i.log env SINGA_AMD_BIAS_INPLACE=0 python bench.py --model bert --steps 30 --warmup 5" || exit $?
done
tools/gpu_step.sh "400 n_sonnx.log python -u tools/bench_suite.py --which bert_sonnx --out gpurun_out/r6/bench_suite_sonnx_r8n.jsonl" || exit $?
