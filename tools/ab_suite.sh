#!/bin/bash
# Alternating A/B of environment settings on tools/bench_suite.py workloads.
# usage: tools/ab_suite.sh OUT.jsonl ROUNDS WHICH "<VAR=val ...>" "<VAR=val ...>" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=$1; shift
R=$1; shift
W=$1; shift
for i in $(seq 1 $R); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python tools/bench_suite.py --which "$W" --steps 20 --warmup 5 > gpurun_out/ab_tmp.log 2>&1 || { echo "bench failed ($cfg)"; tail -5 gpurun_out/ab_tmp.log; exit 1; }
    grep '"bench"' gpurun_out/ab_tmp.log | python3 -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l)
    print(json.dumps({'round': $i, 'env': '$cfg', 'bench': r['bench'], 'value': r['value']}))" | tee -a "$OUT"
  done
done
