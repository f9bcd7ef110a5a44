#!/bin/bash
# Alternating A/B/C... of environment settings on the flagship bench.
# usage: tools/ab_env.sh OUT.jsonl ROUNDS "<VAR=val ...>" "<VAR=val ...>" ...
# (an empty string is the default configuration)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=$1; shift
R=$1; shift
for i in $(seq 1 $R); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ps-parity > gpurun_out/ab_tmp.log 2>&1 || { echo "bench failed ($cfg)"; tail -5 gpurun_out/ab_tmp.log; exit 1; }
    v=$(grep '"metric"' gpurun_out/ab_tmp.log | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['value'])")
    echo "{\"round\": $i, \"env\": \"$cfg\", \"img_s\": $v}" | tee -a "$OUT"
  done
done
