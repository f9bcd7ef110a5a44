#!/bin/bash
# Alternating A/B of the flagship bench between this tree and another checkout
# with its own in-tree build (e.g. a git worktree of an earlier commit).
# usage: tools/ab_tree.sh OUT.jsonl ROUNDS OTHER_DIR
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=$1; R=$2; OTHER=$3
for i in $(seq 1 $R); do
  for t in . "$OTHER"; do
    timeout -k 10 200 python "$t/bench.py" --steps 20 --warmup 5 --no-ps-parity > gpurun_out/ab_tmp.log 2>&1 || { echo "bench failed ($t)"; tail -5 gpurun_out/ab_tmp.log; exit 1; }
    v=$(grep '"metric"' gpurun_out/ab_tmp.log | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['value'])")
    echo "{\"round\": $i, \"tree\": \"$t\", \"img_s\": $v}" | tee -a "$OUT"
  done
done
