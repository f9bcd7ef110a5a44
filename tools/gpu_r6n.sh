#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
S="python tools/bench_suite.py --which bert --out gpurun_out/bert_tiles_r6n.jsonl"
tools/gpu_step.sh "200 c_on1.log env SG_TUNE=14=3 $S" "200 c_t3a.log env SG_TUNE=14=3,4=3 $S" "200 c_t1a.log env SG_TUNE=14=3,4=1 $S" \
  "200 c_on2.log env SG_TUNE=14=3 $S" "200 c_t3b.log env SG_TUNE=14=3,4=3 $S" "200 c_t1b.log env SG_TUNE=14=3,4=1 $S" \
  "200 c_son.log env SG_TUNE=14=3 python tools/bench_suite.py --which bert_sonnx,alexnet --out gpurun_out/bert_tiles_r6n.jsonl" \
  "200 c_soff.log python tools/bench_suite.py --which bert_sonnx,alexnet --out gpurun_out/bert_tiles_r6n.jsonl" \
  "200 c_r50on.log env SG_TUNE=14=3 python bench.py --steps 20 --warmup 5 --no-ps-parity" "200 c_r50off.log python bench.py --steps 20 --warmup 5 --no-ps-parity"
