#!/bin/bash
# PMC passes over the short-K 1x1 convolutions of ResNet-50 at b1024 (forward
# and data gradient): what limits the memory-bound GEMMs.
#   tools/pmc_1x1.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-1x1}
out=gpurun_out/pmc_$tag
mkdir -p $out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P2="FETCH_SIZE GRBM_GUI_ACTIVE"
P3="WRITE_SIZE GRBM_GUI_ACTIVE"
for shp in "64 56 256 fwd" "256 56 64 fwd" "256 14 1024 fwd" "1024 14 256 dgrad" "64 56 256 dgrad"; do
  set -- $shp
  name=c$1_h$2_k$3_$4
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $out/${name}_p$i -o run --output-format csv -- python3 tools/conv_one.py \
      --C $1 --H $2 --K $3 --R 1 --s 1 --batch 1024 --pass $4 --iters 10 > $out/${name}_p$i.log 2>&1 \
      || { echo "pass failed $name p$i rc=$?"; tail -5 $out/${name}_p$i.log; exit 1; }
  done
  echo "done $name"
done
python3 tools/pmc_csv.py $out > $out/summary.txt
