#!/bin/bash
# Whole-step roofline of the flagship ResNet-50 b1024 step: a kernel-trace
# pass (ms per kernel), then PMC passes (HBM bytes read / written per kernel,
# MFMA instruction counts), each its own rocprofv3 run (one counter group per
# pass), summarised by tools/step_roofline.py into gpurun_out/step_roofline_<tag>.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-r5}
out=gpurun_out/roof_$tag
mkdir -p $out
B="python3 bench.py --steps 3 --warmup 2 --no-ps-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format rocpd -- $B > $out/trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 600 rocprofv3 --pmc $P -d $out/pmc$i -o run --output-format rocpd -- $B > $out/pmc$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -5 $out/pmc$i.log; exit 1; }
done
python3 tools/step_roofline.py --steps 5 --trace $(find $out/trace -name '*.db' | head -1) $(find $out/pmc* -name '*.db') > gpurun_out/step_roofline_$tag.txt
rm -rf $out/trace $out/pmc1 $out/pmc2 $out/pmc3
