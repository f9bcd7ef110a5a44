#!/bin/bash
# round 6, call 9o: compile-time GELU forward epilogue: fused-GELU BERT A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  tools/gpu_step.sh "200 o_on$i.log env SINGA_AMD_FUSE_GELU=1 python bench.py --model bert --steps 30 --warmup 5" \
    "200 o_off$i.log python bench.py --model bert --steps 30 --warmup 5" || exit $?
done
