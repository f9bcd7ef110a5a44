#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/prof_step.sh r7f && bash tools/step_roofline.sh r7f
