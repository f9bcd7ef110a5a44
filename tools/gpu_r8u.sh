#!/bin/bash
# round 6, call u: GELU fused into fc1 / fc2 epilogues (now with fc1's bias gradient in fc2's dgrad epilogue): A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
tools/gpu_step.sh "300 u_on1.log env SINGA_AMD_FUSE_GELU=1 python bench.py --model bert --steps 30 --warmup 5" \
  "300 u_off1.log python bench.py --model bert --steps 30 --warmup 5" \
  "300 u_on2.log env SINGA_AMD_FUSE_GELU=1 python bench.py --model bert --steps 30 --warmup 5" \
  "300 u_off2.log python bench.py --model bert --steps 30 --warmup 5" || exit $?
