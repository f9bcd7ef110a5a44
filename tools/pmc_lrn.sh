#!/bin/bash
# LRN timing + two PMC passes (summary -> gpurun_out/pmc_lrn.txt)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_lrn
timeout -k 10 120 python3 tools/lrn_one.py > gpurun_out/lrn_one.jsonl 2>&1 || exit $?
timeout -k 10 120 python3 tools/lrn_one.py --shape 512,256,27,27 >> gpurun_out/lrn_one.jsonl 2>&1 || exit $?
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES"
P2="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_lrn/p$i -o run --output-format csv -- python3 tools/lrn_one.py --iters 3 > gpurun_out/pmc_lrn/p$i.log 2>&1 || { echo "pass failed p=$i rc=$?"; exit 1; }
done
python3 tools/pmc_csv.py gpurun_out/pmc_lrn > gpurun_out/pmc_lrn.txt
