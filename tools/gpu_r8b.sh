#!/bin/bash
# round 6, call b: captured all-reduce pattern probe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SG_LOOP_DEBUG=1
tools/gpu_step.sh "60 p_x1.log python -X faulthandler -u tools/capture_threads_probe.py xrank1 2" && \
tools/gpu_step.sh "60 p_x2.log python -X faulthandler -u tools/capture_threads_probe.py xrank2 2"
