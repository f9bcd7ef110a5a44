#!/bin/bash
# round 6, call w: fused attention backward cost of the bias-gradient sums
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "200 w_fa.log python -u tools/bench_fattn.py" || exit $?
