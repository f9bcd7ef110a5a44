#!/bin/bash
# round 6, call k: native current-stream state + batched attention staging: GPU suite, BERT / sonnx-BERT, ResNet bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "600 t_r8k.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_r8k.log && exit 1
tools/gpu_step.sh "300 k_bert.log python bench.py --model bert --steps 30 --warmup 5" \
  "400 k_suite.log python -u tools/bench_suite.py --which bert_sonnx --out gpurun_out/r6/bench_suite_sonnx_r8k.jsonl" \
  "200 k_r50_1.log python bench.py --steps 20 --warmup 5 --no-ps-parity" "200 k_r50_2.log python bench.py --steps 20 --warmup 5 --no-ps-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pb -o pb --output-format rocpd -- python3 bench.py --model bert --steps 10 --warmup 3 > gpurun_out/pb.log 2>&1 || exit $?
python3 tools/prof_summary.py $(find gpurun_out/pb -name '*.db' | head -1) --steps 13 > gpurun_out/bert_kernel_stats_r8k.txt
rm -rf gpurun_out/pb
