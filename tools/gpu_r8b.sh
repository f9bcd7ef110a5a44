#!/bin/bash
# round 6, call b: captured loopback world, narrowed
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SG_LOOP_DEBUG=1
tools/gpu_step.sh "60 w1.log python -X faulthandler -u tools/world_capture_dbg.py 1" && \
tools/gpu_step.sh "60 w2n.log python -X faulthandler -u tools/world_capture_dbg.py 2 nooverlap" && \
tools/gpu_step.sh "60 w2.log python -X faulthandler -u tools/world_capture_dbg.py 2"
