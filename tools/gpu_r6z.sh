#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 g_e1.log $B" "200 g_g1.log $B --graph" "200 g_e2.log $B" "200 g_g2.log $B --graph" "200 g_e3.log $B" "200 g_g3.log $B --graph"
