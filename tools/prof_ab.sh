#!/bin/bash
# Kernel-trace profiles of the flagship step for the current tree and the
# ab_old/ worktree (an older commit built in place), in one GPU session:
# gpurun_out/prof_{new,old}_<tag>.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-ab}
mkdir -p gpurun_out
for side in new old; do
  dir=.
  [ $side = old ] && dir=ab_old
  out=$GRAFT_REPO_ROOT/gpurun_out/prof_${side}_$tag
  (cd $dir && timeout -k 10 300 rocprofv3 --kernel-trace -d $out -o r50 --output-format rocpd -- python3 bench.py --steps 8 --warmup 3 --no-ps-parity > $out.log 2>&1) || exit $?
  db=$(find $out -name '*.db' | head -1)
  python3 tools/prof_summary.py "$db" --steps 11 > $out.txt
  rm -rf $out
done
