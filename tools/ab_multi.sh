#!/bin/bash
# A/B/C... of tuning-knob settings on the flagship bench, alternating rounds.
# usage: tools/ab_multi.sh rounds "<SG_TUNE 1>" "<SG_TUNE 2>" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
R=$1; shift
for i in $(seq 1 $R); do
  for cfg in "$@"; do
    SG_TUNE="$cfg" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ps-parity > gpurun_out/ab_tmp.log 2>&1 || { echo "bench failed ($cfg)"; tail -5 gpurun_out/ab_tmp.log; exit 1; }
    v=$(grep '"metric"' gpurun_out/ab_tmp.log | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['value'])")
    echo "{\"round\": $i, \"SG_TUNE\": \"$cfg\", \"img_s\": $v}" | tee -a gpurun_out/ab_multi.jsonl
  done
done
