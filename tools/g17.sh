tools/gpu_step.sh \
 "900 gputests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 smoke.log python -c 'import __graft_entry__ as g; g.smoke()'" \
 "600 bench.log python bench.py --steps 30 --warmup 10"
