tools/gpu_step.sh \
 "300 kt.log python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "300 tw5.log python tools/tune_conv.py --batch 256 --knob 0 --values 5,4 --pass wgrad" \
 "300 tdx.log python tools/tune_conv.py --batch 256 --knob 1 --values 1 --pass dx" \
 "300 bench_b256.log python bench.py --steps 30 --warmup 5" \
 "300 bench_b512.log python bench.py --steps 20 --warmup 5 --batch 512"
