#!/bin/bash
# round 6, call c: GPU suite, bench N=1 x2, loopback rehearsals, alexnet / bert, GEMM per-shape profile
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "600 t_r8c.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "200 c_1.log $B" "200 c_2.log $B" \
  "300 c_loop2.log python bench.py --gpus 2 --loopback --batch 128 --steps 3 --warmup 3" \
  "300 c_loop4.log python bench.py --gpus 4 --loopback --batch 64 --steps 3 --warmup 3" || exit $?
export SG_GEMM_LOG=1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gs -o gs --output-format rocpd -- python3 bench.py --eager --steps 2 --warmup 1 --no-ps-parity > gpurun_out/gs.log 2> gpurun_out/gemm.log || exit $?
unset SG_GEMM_LOG
python3 tools/gemm_shapes.py $(find gpurun_out/gs -name '*.db' | head -1) gpurun_out/gemm.log --steps 3 > gpurun_out/gemm_shapes.txt
rm -rf gpurun_out/gs
