#!/bin/bash
# PMC passes over the fwd / dgrad / wgrad kernels of one conv shape.
# usage: tools/pmc_pass.sh <tag> "<passes>" <conv_one args...>   e.g. tools/pmc_pass.sh c3 "fwd wgrad" --C 256 --H 14
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
passes=$1; shift
mkdir -p gpurun_out/pmc_$tag
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
for ps in $passes; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_$tag/${ps}_p$i -o run --output-format csv -- python3 tools/conv_one.py --pass $ps "$@" > gpurun_out/pmc_$tag/${ps}_p$i.log 2>&1 || { echo "pass failed $ps p=$i rc=$?"; exit 1; }
  done
done
python3 tools/pmc_csv.py gpurun_out/pmc_$tag > gpurun_out/pmc_$tag.txt
