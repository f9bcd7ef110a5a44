#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 workq_r5i.log python -u -m pytest tests/test_workq_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "300 workq_static_r5i.log env SG_WORKQ=0 python -u -m pytest tests/test_workq_gpu.py -x -v -k stress --timeout 120 --timeout-method thread" \
  "300 bert_r5i.log python tools/bert_vs_torch.py --size tiny --steps 8" \
  "300 bertbase_r5i.log python tools/bert_vs_torch.py --size base --steps 6"
