cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "600 gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" "300 suite.log python tools/bench_suite.py --which bert,bert_sonnx --steps 20 --warmup 5" || exit $?
bash tools/alexnet_timeline.sh
