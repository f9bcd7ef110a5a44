#!/bin/bash
# GPU tests (all, or those matching $1) then the AlexNet kernel profile + suite.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
sel=${1:+-k $1}
tools/gpu_step.sh "600 gputest.log python -u -m pytest tests -m gpu $sel -x -q --timeout 120 --timeout-method thread" && bash tools/alexnet_prof.sh
