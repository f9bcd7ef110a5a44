#!/bin/bash
# PMC passes over one plain GEMM shape under several tile policies.
# usage: tools/pmc_gemm.sh <tag> "<policies>" <gemm_one args...>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
pols=$1; shift
mkdir -p gpurun_out/pmc_$tag
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
P4="WRITE_SIZE"
for pol in $pols; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_$tag/p${pol}_$i -o run --output-format csv -- python3 tools/gemm_one.py --policy $pol "$@" > gpurun_out/pmc_$tag/p${pol}_$i.log 2>&1 || { echo "pass failed pol=$pol p=$i rc=$?"; exit 1; }
  done
done
python3 tools/pmc_csv.py gpurun_out/pmc_$tag > gpurun_out/pmc_$tag.txt
