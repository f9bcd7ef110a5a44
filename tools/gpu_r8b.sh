#!/bin/bash
# round 6, call b: step trace of the captured loopback world
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SG_LOOP_DEBUG=1
tools/gpu_step.sh "120 dbg_world.log python -X faulthandler -u tools/world_capture_dbg.py 2"
