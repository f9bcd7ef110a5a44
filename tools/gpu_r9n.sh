#!/bin/bash
# round 6, call 9n: PMC passes over tools/bench_actgrad.py (plain / act-grad / beta-1 epilogues)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
rm -rf gpurun_out/pmc/*
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM SQ_WAIT_INST_ANY -d gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 tools/bench_actgrad.py --iters 5 > gpurun_out/pmc/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 tools/bench_actgrad.py --iters 5 > gpurun_out/pmc/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc/p3 -o p3 --output-format csv -- python3 tools/bench_actgrad.py --iters 5 > gpurun_out/pmc/p3.log 2>&1 || exit $?
