#!/bin/bash
# Instruction-mix PMC pass (per-wave instruction classes) over one conv pass.
# usage: tools/pmc_inst.sh <tag> <pass> <conv_one args...>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
ps=$1; shift
mkdir -p gpurun_out/pmc_$tag
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmc_$tag/${ps}_i -o run --output-format csv -- python3 tools/conv_one.py --pass $ps "$@" > gpurun_out/pmc_$tag/${ps}_i.log 2>&1 || { echo "pass failed rc=$?"; exit 1; }
python3 tools/pmc_csv.py gpurun_out/pmc_$tag > gpurun_out/pmc_$tag.txt
