#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tools/gpu_step.sh "300 gt_wdot.log python -u -m pytest tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k identity_sum" || exit 1
SINGA_AMD_BN_WDOT=1 bash tools/prof_step.sh wdot1
