#!/bin/bash
# Instruction-mix, stall and LDS PMC passes over the persistent stage-1 3x3
# conv (csrc/kernels/conv3x3.hip), forward and data gradient.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_c3
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P3="SQ_WAIT_INST_LDS SQ_INSTS_WAVE32_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
for ps in fwd dgrad; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_c3/${ps}_p$i -o run --output-format csv -- python3 tools/bench_conv3x3.py --only $ps --iters 5 > gpurun_out/pmc_c3/${ps}_p$i.log 2>&1 || { echo "pass failed $ps $i rc=$?"; exit 1; }
  done
done
python3 tools/pmc_csv.py gpurun_out/pmc_c3 > gpurun_out/pmc_c3.txt
