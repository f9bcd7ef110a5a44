tools/gpu_step.sh \
 "400 bench_b768.log python bench.py --steps 20 --warmup 8 --batch 768" \
 "400 bench_b1024.log python bench.py --steps 20 --warmup 8 --batch 1024"
