#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "400 t_r7i.log python -u -m pytest tests/test_bnres_gpu.py tests/test_models_gpu.py -q -k 'bnres or tail or resnet or bottleneck' --timeout 120 --timeout-method thread -p no:cacheprovider" && \
B="python bench.py --steps 20 --warmup 5 --no-ps-parity"
tools/gpu_step.sh "200 i_1.log $B" "200 i_2.log $B" "200 i_3.log $B" && bash tools/prof_step.sh r7i
