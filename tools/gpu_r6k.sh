#!/bin/bash
# full GPU suite, no early stop
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "1100 gputests_r6k.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider"
