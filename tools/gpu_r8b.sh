#!/bin/bash
# round 6, call b: which capture patterns does hipStreamEndCapture survive?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SG_LOOP_DEBUG=1
tools/gpu_step.sh "60 p_fj.log python -X faulthandler -u tools/capture_threads_probe.py forkjoin 1" && \
tools/gpu_step.sh "60 p_mf.log python -X faulthandler -u tools/capture_threads_probe.py multifork 1" && \
tools/gpu_step.sh "60 p_ch.log python -X faulthandler -u tools/capture_threads_probe.py chain 1" && \
tools/gpu_step.sh "60 p_ne.log python -X faulthandler -u tools/capture_threads_probe.py nested 1"
