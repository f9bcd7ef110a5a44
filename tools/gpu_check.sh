#!/bin/bash
# One GPU session: GPU tests, the flagship bench, and a rocprofv3 kernel-stats
# profile of the bench step.  usage: tools/gpu_check.sh TAG [pytest -k expr]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-run}
K=${2:-}
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KA[@]}" \
  > gpurun_out/gputest_$TAG.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
tail -2 gpurun_out/gputest_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
grep metric gpurun_out/bench_$TAG.log
bash tools/prof_step.sh "$TAG" || { echo "profile failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
head -30 gpurun_out/prof_$TAG.txt
