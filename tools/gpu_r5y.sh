#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kd -o r50 --output-format rocpd -- python3 bench.py --steps 3 --warmup 2 --no-ps-parity > gpurun_out/kd.log 2>&1 || exit $?
db=$(find gpurun_out/kd -name '*.db' | head -1)
for k in "igemm_k<128, 128, 0, 0, 0, 256, 2, 2, 1, 0>" "igemm_k<128, 128, 1, 4, 2, 512, 2, 4, 2, 0>" "igemm_k<128, 128, 2, 0, 0, 512" "igemm_k<128, 128, 3, 6, 0, 512" "bn_bwd_apply_k" "bn_apply_kIDF16bLi8ELi1ELb0ELb0E"; do
  echo "== $k"; python3 tools/kernel_dispatches.py "$db" "$k" --steps 5
done > gpurun_out/kd_r5y.txt
rm -rf gpurun_out/kd
