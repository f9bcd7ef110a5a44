tools/gpu_step.sh \
 "600 bench_default.log python bench.py" \
 "600 bench_default2.log python bench.py --steps 30 --warmup 10"
