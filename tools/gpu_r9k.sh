#!/bin/bash
# round 6 end: full GPU suite + smoke + default bench on the final tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "700 t_end.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_end.log && exit 1
tools/gpu_step.sh "200 k_smoke.log python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" "200 k_r50.log python bench.py" || exit $?
