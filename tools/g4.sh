tools/gpu_step.sh \
 "300 kt.log python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "300 tune_wgrad2.log python tools/tune_conv.py --batch 256 --knob 0 --values 4,0,1 --pass wgrad" \
 "300 bench_b256.log python bench.py --steps 30 --warmup 5"
