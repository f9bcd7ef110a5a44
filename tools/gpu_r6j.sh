#!/bin/bash
# full GPU test suite + smoke on the current build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "1100 gputests_r6j.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" && \
tools/gpu_step.sh "200 smoke_r6j.log python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
