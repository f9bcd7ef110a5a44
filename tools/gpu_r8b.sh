#!/bin/bash
# round 6, call b: cross-thread capture probe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "60 p_single.log python -X faulthandler -u tools/capture_threads_probe.py single 2" && \
tools/gpu_step.sh "60 p_tempev.log python -X faulthandler -u tools/capture_threads_probe.py tempev 2" && \
tools/gpu_step.sh "60 p_launchB.log python -X faulthandler -u tools/capture_threads_probe.py launchB 2" && \
tools/gpu_step.sh "60 p_forkB.log python -X faulthandler -u tools/capture_threads_probe.py forkB 2"
