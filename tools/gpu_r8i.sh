#!/bin/bash
# round 6, call i: current-build step profile (kernel stats + purity) and whole-step roofline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/prof_step.sh r8i || exit $?
bash tools/step_roofline.sh r8i
