#!/bin/bash
# round 6, call p: sonnx import with the bf16 residual stream: tests + sonnx-BERT bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "300 t_sonnx.log python -u -m pytest tests/test_models_gpu.py -k 'sonnx or bert' -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -s" || exit $?
grep -q "failed" gpurun_out/t_sonnx.log && exit 1
tools/gpu_step.sh "400 p_sonnx1.log python -u tools/bench_suite.py --which bert_sonnx --out gpurun_out/r6/bench_suite_sonnx_r8p.jsonl" \
  "400 p_sonnx2.log python -u tools/bench_suite.py --which bert_sonnx --out gpurun_out/r6/bench_suite_sonnx_r8p.jsonl" \
  "400 ls_sonnx2.log python -u tools/launch_sites.py --model bert_sonnx --batch 32 --top 60" || exit $?
