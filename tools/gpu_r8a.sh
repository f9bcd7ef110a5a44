#!/bin/bash
# round 6, call a: GPU suite (incl. captured multi-rank world, workq arenas),
# bench N=1 x2, loopback rehearsal of the N>1 captured path, alexnet / bert via bench.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "600 t_r8a.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" && \
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 a_1.log $B" "200 a_2.log $B" \
  "300 a_loop2.log python bench.py --gpus 2 --loopback --batch 128 --steps 3 --warmup 3" \
  "300 a_loop4.log python bench.py --gpus 4 --loopback --batch 64 --steps 3 --warmup 3" \
  "300 a_alex.log python bench.py --model alexnet --steps 20 --warmup 5" \
  "300 a_bert.log python bench.py --model bert --steps 20 --warmup 5"
cd "$GRAFT_REPO_ROOT" && export SG_GEMM_LOG=1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gs -o gs --output-format rocpd -- python3 bench.py --eager --steps 2 --warmup 1 --no-ps-parity > gpurun_out/gs.log 2> gpurun_out/gemm.log && \
unset SG_GEMM_LOG && python3 tools/gemm_shapes.py $(find gpurun_out/gs -name '*.db' | head -1) gpurun_out/gemm.log --steps 3 > gpurun_out/gemm_shapes.txt; rm -rf gpurun_out/gs
