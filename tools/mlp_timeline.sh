#!/bin/bash
# One-step dispatch timeline of the fp32 MLP (mlp_gpu bench) -> gpurun_out/mlp_timeline.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/mlp_tl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/mlp_tl -o k --output-format rocpd -- \
  python3 tools/bench_suite.py --which mlp_gpu --steps 3 --warmup 2 "$@" > gpurun_out/mlp_tl.log 2>&1 || exit 1
db=$(find gpurun_out/mlp_tl -name '*.db' | head -1)
python3 tools/step_timeline.py "$db" > gpurun_out/mlp_timeline.txt && rm -rf gpurun_out/mlp_tl
