#!/bin/bash
# 3-stage ring (knob 14) : correctness under the knob, BERT suite A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 t_ring_r6m.log env SG_TUNE=14=3 python -u -m pytest tests/test_kernels_gpu.py tests/test_bert_fused_gpu.py tests/test_models_gpu.py -q -k 'gemm or matmul or bert or linear or attention' --timeout 120 --timeout-method thread -p no:cacheprovider" && \
S="python tools/bench_suite.py --which bert --out gpurun_out/bert_ring_r6m.jsonl"
tools/gpu_step.sh "200 b_off1.log $S" "200 b_on1.log env SG_TUNE=14=3 $S" "200 b_off2.log $S" "200 b_on2.log env SG_TUNE=14=3 $S" \
  "200 b_off3.log $S" "200 b_on3.log env SG_TUNE=14=3 $S" && \
tools/gpu_step.sh "300 prof_bert_ring.log env SG_TUNE=14=3 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o bert --output-format rocpd -- python3 tools/bench_suite.py --which bert --steps 10 --warmup 3 --no-graph" || exit $?
db=$(find gpurun_out/prof_bert -name '*.db' | head -1)
python3 tools/prof_summary.py "$db" --steps 13 > gpurun_out/prof_bert_ring_r6m.txt
python3 tools/kernel_dispatches.py "$db" "igemm_k" --steps 13 > gpurun_out/bert_dispatch_ring_r6m.txt
rm -rf gpurun_out/prof_bert
