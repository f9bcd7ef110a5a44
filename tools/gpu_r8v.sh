#!/bin/bash
# round 6, call v: full GPU suite + smoke + bench set + BERT kernel stats on the current build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "700 t_r8v.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_r8v.log && exit 1
tools/gpu_step.sh "200 v_smoke.log python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "200 v_r50.log python bench.py" \
  "300 v_mlp.log python -u tools/bench_suite.py --which mlp_gpu --out gpurun_out/r6/bench_suite_r8v.jsonl" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pb -o pb --output-format rocpd -- python3 bench.py --model bert --steps 10 --warmup 3 > gpurun_out/pb.log 2>&1 || exit $?
python3 tools/prof_summary.py $(find gpurun_out/pb -name '*.db' | head -1) --steps 13 > gpurun_out/r6/bert_b32s128_kernel_stats_r8v.txt
rm -rf gpurun_out/pb
