#!/bin/bash
# round 6, call b: captured all-reduce pattern probe, reduction on the origin stream
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "60 p_o1.log python -X faulthandler -u tools/capture_threads_probe.py xorig1 2" && \
tools/gpu_step.sh "60 p_o2.log python -X faulthandler -u tools/capture_threads_probe.py xorig2 2"
