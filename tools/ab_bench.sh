#!/bin/bash
# A/B of a tuning knob on the flagship bench: alternating runs in one box.
# usage: tools/ab_bench.sh "<SG_TUNE for A>" "<SG_TUNE for B>" [rounds]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A=$1; B=$2; R=${3:-2}
for i in $(seq 1 $R); do
  for cfg in "$A" "$B"; do
    SG_TUNE="$cfg" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ps-parity > gpurun_out/ab_tmp.log 2>&1 || { echo "bench failed ($cfg)"; tail -5 gpurun_out/ab_tmp.log; exit 1; }
    v=$(grep '"metric"' gpurun_out/ab_tmp.log | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['value'])")
    echo "{\"round\": $i, \"SG_TUNE\": \"$cfg\", \"img_s\": $v}" | tee -a gpurun_out/ab.jsonl
  done
done
