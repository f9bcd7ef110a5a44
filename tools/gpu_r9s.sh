#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_9s.log python -u -m pytest tests/test_bnres_gpu.py -k gram -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
