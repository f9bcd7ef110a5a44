#!/bin/bash
# round 6, call b: the crash of test_captured_distopt_world (faulthandler), then the rest of the suite
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "240 t_cap.log python -X faulthandler -u -m pytest tests/test_captured_world_gpu.py -x -v -s -p no:cacheprovider -k 'world and False-2'"
