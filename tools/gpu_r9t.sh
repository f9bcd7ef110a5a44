#!/bin/bash
# round 6: GEMM knob re-check on the final BERT step (knob 14: three-stage ring policy; knob 6: short-K cap)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "" "14=3" "14=-1" "6=4" "" "14=3"; do
  tools/gpu_step.sh "200 t_knob_${spec//[=,-]/_}_$RANDOM.log env SG_TUNE=$spec python bench.py --model bert --steps 30 --warmup 5" || exit $?
done
