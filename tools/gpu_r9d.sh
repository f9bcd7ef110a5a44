#!/bin/bash
# round 6 final: full GPU suite, smoke, bench set, ResNet-50 kernel stats (rocprofv3 --stats) into profiles
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "700 t_final.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_final.log && exit 1
tools/gpu_step.sh "200 f_smoke.log python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "200 f_r50_1.log python bench.py" "200 f_r50_2.log python bench.py --steps 20 --warmup 5" \
  "200 f_alex.log python bench.py --model alexnet --steps 30 --warmup 5" \
  "200 f_bert.log python bench.py --model bert --steps 30 --warmup 5" \
  "400 f_suite.log python -u tools/bench_suite.py --which bert_sonnx,mlp_gpu --out gpurun_out/r6/bench_suite_final.jsonl" || exit $?
rm -rf gpurun_out/pf
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pf -o r50 --output-format rocpd -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/pf.log 2>&1 || exit $?
DB=$(find gpurun_out/pf -name 'r50_results.db' | head -1)
python3 tools/step_kernels.py $DB > gpurun_out/r6/r50_step_kernels_final.txt
python3 tools/timeline_gaps.py $DB --last 6 --min-kernels 300 > gpurun_out/r6/timeline_gaps_resnet50_final.txt
find gpurun_out/pf -name '*kernel_stats.csv' -exec cp {} gpurun_out/r6/r50_kernel_stats_final.csv \;
rm -rf gpurun_out/pf
