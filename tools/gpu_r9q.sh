#!/bin/bash
# round 6 final: step profile (kernel stats + purity) and whole-step roofline of the final build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/prof_step.sh r9q || exit $?
bash tools/step_roofline.sh r9q
