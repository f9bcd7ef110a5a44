#!/bin/bash
# PMC passes over fp32 generic-GEMM configurations (ggemm.hip).
# usage: tools/pmc_ggemm.sh <tag> "<name:gemm_one args>"...   (args use commas for spaces)
#   e.g. tools/pmc_ggemm.sh f32 "sq:--M,4096,--N,4096,--K,4096,--tile,1" "mlp:--M,1024,--N,2000,--K,2500,--kout"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/pmc_$tag
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
P3="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_CYCLES"
for spec in "$@"; do
  name=${spec%%:*}
  args=${spec#*:}
  args=${args//,/ }
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_$tag/${name}_$i -o run --output-format csv -- \
      python3 tools/gemm_one.py --f32 $args > gpurun_out/pmc_$tag/${name}_$i.log 2>&1 || { echo "pass failed $name p=$i rc=$?"; exit 1; }
  done
done
python3 tools/pmc_csv.py gpurun_out/pmc_$tag > gpurun_out/pmc_$tag.txt
