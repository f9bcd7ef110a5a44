#!/bin/bash
# round 6, call g: streaming 1x1 GEMM (knob 18): tests, per-shape map, step A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "300 t_st.log python -u -m pytest tests/test_stgemm_gpu.py tests/test_workq_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_st.log && exit 1
tools/gpu_step.sh "300 g_1x1.log python -u tools/bench_1x1.py --policies default,stream --out gpurun_out/r6/bench_1x1_stream.jsonl" \
  "200 g_off1.log $B" "200 g_on1.log SG_TUNE=18=1 $B" "200 g_off2.log $B" "200 g_on2.log SG_TUNE=18=1 $B"
