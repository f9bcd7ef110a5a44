#!/bin/bash
# round 6, call l: attention staging with unconditional loads: tests + BERT / sonnx-BERT + kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "300 t_fa.log python -u -m pytest tests/test_fattn_gpu.py tests/test_bert_fused_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_fa.log && exit 1
tools/gpu_step.sh "300 l_bert1.log python bench.py --model bert --steps 30 --warmup 5" "300 l_bert2.log python bench.py --model bert --steps 30 --warmup 5" \
  "400 l_sonnx.log python -u tools/bench_suite.py --which bert_sonnx --out gpurun_out/r6/bench_suite_sonnx_r8l.jsonl" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pb -o pb --output-format rocpd -- python3 bench.py --model bert --steps 10 --warmup 3 > gpurun_out/pb.log 2>&1 || exit $?
python3 tools/prof_summary.py $(find gpurun_out/pb -name '*.db' | head -1) --steps 13 > gpurun_out/bert_kernel_stats_r8l.txt
rm -rf gpurun_out/pb
