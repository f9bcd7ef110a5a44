#!/bin/bash
# fp32 LDS-DMA GEMM: exactness tests, then the MLP shape sweep (DMA on/off)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

tools/gpu_step.sh "400 gg_sweep_r6g.log python tools/bench_ggemm_f32.py --tiles 1,3,4,5,7 --splits=-1,2,3 --out gpurun_out/gg_sweep_r6g.jsonl" && \
tools/gpu_step.sh "200 mlp_r6g.log python tools/bench_suite.py --which mlp_gpu"
