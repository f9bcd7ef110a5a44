#!/bin/bash
# secondary configs on the current build + AlexNet kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 suite_r6f.log python tools/bench_suite.py --which mlp_gpu,alexnet,bert,bert_sonnx --out gpurun_out/bench_suite_r6f.jsonl" && \
tools/gpu_step.sh "300 alex_prof_r6f.log bash tools/alexnet_prof.sh r6f"
