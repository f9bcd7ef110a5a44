#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
S="python tools/bench_suite.py --which alexnet"
tools/gpu_step.sh "200 a_on1.log $S" "200 a_off1.log env SG_TUNE=15=0 $S" "200 a_on2.log $S" "200 a_off2.log env SG_TUNE=15=0 $S" "200 a_k6.log env SG_TUNE=6=8 $S" "200 a_k14.log env SG_TUNE=14=-1 $S"
