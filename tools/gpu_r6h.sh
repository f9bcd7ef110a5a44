#!/bin/bash
# fp32 GEMM with the DMA-aware tile picker: tests, sweep (auto only + DMA tiles), MLP suite x2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_gg_r6h.log python -u -m pytest tests/test_generic_gemm_gpu.py tests/test_models_gpu.py -x -q -k 'fp32 or mlp or gemm' --timeout 120 --timeout-method thread" && \
tools/gpu_step.sh "400 gg_sweep_r6h.log python tools/bench_ggemm_f32.py --tiles 1,7 --splits=-1,3 --dma 0 --out gpurun_out/gg_sweep_r6h.jsonl" && \
tools/gpu_step.sh "200 mlp_r6h_1.log python tools/bench_suite.py --which mlp_gpu" "200 mlp_r6h_2.log python tools/bench_suite.py --which mlp_gpu --out gpurun_out/mlp_r6h.jsonl"
