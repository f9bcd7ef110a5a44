#!/bin/bash
# round 6, call 9f: BERT timed-step kernel table
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
rm -rf gpurun_out/pb
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pb -o bert --output-format rocpd -- python3 bench.py --model bert --steps 10 --warmup 3 > gpurun_out/pb.log 2>&1 || exit $?
python3 tools/step_kernels.py $(find gpurun_out/pb -name 'bert_results.db' | head -1) --min 250 --max 400 > gpurun_out/r6/bert_step_kernels_r9f.txt
rm -rf gpurun_out/pb
