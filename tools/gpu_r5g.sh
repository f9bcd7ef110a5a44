#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3 4 5 6; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ps-parity > gpurun_out/benchR${i}_r5g.log 2>&1
  rc=$?; echo "run $i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
done
exit 0
