#!/bin/bash
# round 6, call b: captured loopback world on one stream
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SG_LOOP_DEBUG=1
tools/gpu_step.sh "60 w2.log python -X faulthandler -u tools/world_capture_dbg.py 2" && \
tools/gpu_step.sh "60 w4.log python -X faulthandler -u tools/world_capture_dbg.py 4"
