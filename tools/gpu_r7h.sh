#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 h_base1.log $B" "200 h_c3.log env SINGA_AMD_CONV3X3=0 $B" "200 h_rpt2.log env SINGA_BN_RPT=2 $B" "200 h_rpt8.log env SINGA_BN_RPT=8 $B" "200 h_base2.log $B" "200 h_bucket.log env SG_TUNE=12=0 $B"
