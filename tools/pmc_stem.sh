#!/bin/bash
# Instruction-mix and stall PMC passes over the paired-tap stem conv.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_stem
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for ps in fwd wgrad; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_stem/${ps}_p$i -o run --output-format csv -- python3 tools/stem_one.py --pass $ps > gpurun_out/pmc_stem/${ps}_p$i.log 2>&1 || { echo "pass failed $ps $i rc=$?"; exit 1; }
  done
done
python3 tools/pmc_csv.py gpurun_out/pmc_stem > gpurun_out/pmc_stem.txt
