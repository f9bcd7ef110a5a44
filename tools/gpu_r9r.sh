#!/bin/bash
# round 6 final: secondary configs on the final build (BERT step kernels, sonnx-BERT, AlexNet, MLP)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "200 r_alex.log python bench.py --model alexnet --steps 30 --warmup 5" "200 r_bert.log python bench.py --model bert --steps 30 --warmup 5" \
  "400 r_suite.log python -u tools/bench_suite.py --which bert_sonnx,mlp_gpu --out gpurun_out/r6/bench_suite_final_r9r.jsonl" || exit $?
rm -rf gpurun_out/pb
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pb -o bert --output-format rocpd -- python3 bench.py --model bert --steps 10 --warmup 3 > gpurun_out/pb.log 2>&1 || exit $?
python3 tools/step_kernels.py $(find gpurun_out/pb -name 'bert_results.db' | head -1) --min 250 --max 400 > gpurun_out/r6/bert_step_kernels_final.txt
rm -rf gpurun_out/pb
