tools/gpu_step.sh \
 "600 tests_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "240 smoke.log python -c 'import __graft_entry__ as g; g.smoke()'" \
 "300 bench_graph.log python bench.py --steps 30 --warmup 5" \
 "300 bench_eager.log python bench.py --steps 20 --warmup 5 --no-graph"
