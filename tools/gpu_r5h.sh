#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 workq_r5h.log python -u -m pytest tests/test_workq_gpu.py -x -q --timeout 120 --timeout-method thread" || exit $?
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ps-parity > gpurun_out/benchR${i}_r5h.log 2>&1
  rc=$?; echo "run $i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
done
bash tools/prof_step.sh r5h && bash tools/step_roofline.sh r5h
