tools/gpu_step.sh \
 "300 bench_b384.log python bench.py --steps 20 --warmup 5 --batch 384" \
 "300 bench_b512.log python bench.py --steps 20 --warmup 5 --batch 512" \
 "300 tune_wgrad.log python tools/tune_conv.py --batch 256 --knob 0 --values 4,0,1,2,3 --pass wgrad" \
 "300 tune_fwd.log python tools/tune_conv.py --batch 256 --knob 1 --values 1 --pass fwd" \
 "300 tune_dgrad.log python tools/tune_conv.py --batch 256 --knob 1 --values 1 --pass dgrad" \
 "120 ps1.log python tools/ps_bench.py --iters 200"
