#!/bin/bash
# MLP: DMA tile filter (default) vs unrestricted pick, alternating on one box; then the final-build step roofline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
S="python tools/bench_suite.py --which mlp_gpu --out gpurun_out/mlp_ab_r6i.jsonl"
tools/gpu_step.sh "200 mlp_f1.log $S" "200 mlp_u1.log env SG_GG_TUNE=2=1 $S" "200 mlp_n1.log env SG_GG_TUNE=2=-1 $S" \
  "200 mlp_f2.log $S" "200 mlp_u2.log env SG_GG_TUNE=2=1 $S" "200 mlp_n2.log env SG_GG_TUNE=2=-1 $S" \
  "200 mlp_f3.log $S" "200 mlp_u3.log env SG_GG_TUNE=2=1 $S" && \
bash tools/step_roofline.sh r6i
