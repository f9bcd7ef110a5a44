#!/bin/bash
# dispatch shapes of the top generic kernels on the final build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v -o r50 --output-format rocpd -- python3 bench.py --steps 8 --warmup 3 --no-ps-parity > gpurun_out/prof_v.log 2>&1 || exit $?
db=$(find gpurun_out/prof_v -name '*.db' | head -1)
: > gpurun_out/dispatch_v.txt
for k in "igemm_k<128, 128, 0, 0, 0, 256, 2, 2, 1, 0>" "igemm_k<128, 128, 7, 0, 0, 512" "igemm_k<128, 128, 2, 0, 0, 512" "igemm_k<128, 128, 3, 6, 0, 512" "igemm_k<128, 128, 0, 0, 0, 512" "igemm_k<128, 64, 0, 0, 0, 256" "bn_bwd_apply_k" "bn_apply_kIDF16bLi8ELi1ELb0ELb0E"; do
  echo "== $k" >> gpurun_out/dispatch_v.txt
  python3 tools/kernel_dispatches.py "$db" "$k" --steps 11 >> gpurun_out/dispatch_v.txt
done
rm -rf gpurun_out/prof_v
