tools/gpu_step.sh \
 "400 t_all.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "300 bench_b256.log python bench.py --steps 30 --warmup 5" \
 "300 bench_b512.log python bench.py --steps 20 --warmup 5 --batch 512"
