#!/bin/bash
# round 6, call 9m: unconditional loads in the LayerNorm kernels: tests, BERT benches, step kernels
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "400 t_9m.log python -u -m pytest tests/test_bert_fused_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -k 'layernorm or drop_add or bert or sonnx or norm' -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_9m.log && exit 1
tools/gpu_step.sh "200 m_bert1.log python bench.py --model bert --steps 30 --warmup 5" "200 m_bert2.log python bench.py --model bert --steps 30 --warmup 5" || exit $?
rm -rf gpurun_out/pb
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pb -o bert --output-format rocpd -- python3 bench.py --model bert --steps 10 --warmup 3 > gpurun_out/pb.log 2>&1 || exit $?
python3 tools/step_kernels.py $(find gpurun_out/pb -name 'bert_results.db' | head -1) --min 250 --max 400 > gpurun_out/r6/bert_step_kernels_r9m.txt
rm -rf gpurun_out/pb
