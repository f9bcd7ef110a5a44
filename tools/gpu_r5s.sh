#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_sonnx_r5s.log python -u -m pytest tests -m gpu -x -q -k 'sonnx or bert' --timeout 120 --timeout-method thread" \
  "300 suite_r5s.log python tools/bench_suite.py --which bert_sonnx,bert --steps 20 --warmup 5"
