#!/bin/bash
# Kernel profiles of the flagship step under two environments on ONE box:
#   tools/prof_ab.sh <tag> "<env assignments A>" "<env assignments B>"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1
for side in A B; do
  if [ $side = A ]; then envs=$2; else envs=$3; fi
  ( export $envs; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_$side -o r50 --output-format rocpd -- python3 bench.py --steps 8 --warmup 3 --no-ps-parity > gpurun_out/prof_${tag}_$side.log 2>&1 ) || exit $?
  db=$(find gpurun_out/prof_${tag}_$side -name '*.db' | head -1)
  python3 tools/prof_summary.py "$db" --steps 11 > gpurun_out/prof_${tag}_$side.txt
  rm -rf gpurun_out/prof_${tag}_$side
done
