#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 f_suite.log python tools/bench_suite.py --which mlp_gpu,alexnet,bert,bert_sonnx,mlp_cpu --out gpurun_out/bench_suite_final_r7c.jsonl" \
  "200 f_b1.log python bench.py" "200 f_b2.log python bench.py"
