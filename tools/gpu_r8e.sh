#!/bin/bash
# round 6, call e: 8-wave fused attention + BERT A/B + GEMM per-shape profile (greedy join)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BB="python bench.py --model bert --steps 30 --warmup 5"
tools/gpu_step.sh "300 t_fa.log python -u -m pytest tests/test_fattn_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_fa.log && exit 1
tools/gpu_step.sh "200 e_bert_f1.log $BB" "200 e_bert_u1.log SINGA_AMD_FATTN=0 $BB" "200 e_bert_f2.log $BB" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pb -o pb --output-format rocpd -- python3 bench.py --model bert --steps 10 --warmup 3 > gpurun_out/pb.log 2>&1 || exit $?
python3 tools/prof_summary.py $(find gpurun_out/pb -name '*.db' | head -1) --steps 13 > gpurun_out/bert_kernel_stats_fattn8.txt
rm -rf gpurun_out/pb
export SG_GEMM_LOG=1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gs -o gs --output-format rocpd -- python3 bench.py --eager --steps 2 --warmup 1 --no-ps-parity > gpurun_out/gs.log 2> gpurun_out/gemm.log || exit $?
unset SG_GEMM_LOG
python3 tools/gemm_shapes.py $(find gpurun_out/gs -name '*.db' | head -1) gpurun_out/gemm.log --steps 3 > gpurun_out/gemm_shapes.txt
rm -rf gpurun_out/gs
