#!/bin/bash
# round 6, call j: b256 bench, suite (sonnx-BERT / BERT / MLP GPU / AlexNet), torch-call report
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "200 j_b256.log python bench.py --batch 256 --steps 30 --warmup 5 --no-ps-parity" \
  "600 j_suite.log python -u tools/bench_suite.py --which mlp_gpu,bert,bert_sonnx,alexnet --out gpurun_out/r6/bench_suite_r6.jsonl" \
  "600 j_tc.log python -u tools/torch_calls.py --which resnet50,bert,mlp_gpu"
