#!/bin/bash
# round 6, call 9c: LayerNorm backward rows per wave (SG_LNB_RPW) on BERT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_9c.log python -u -m pytest tests/test_bert_fused_gpu.py tests/test_kernels_gpu.py -k 'layernorm or drop_add or bert' -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_9c.log && exit 1
for r in 4 1 2 8 4 1 2; do
  tools/gpu_step.sh "200 c_rpw$r.$RANDOM.log env SG_LNB_RPW=$r python bench.py --model bert --steps 30 --warmup 5" || exit $?
done
