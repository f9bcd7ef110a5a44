tools/gpu_step.sh \
 "400 kt12.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "300 tdx5.log python tools/tune_conv.py --batch 256 --knob 5 --values 0,1 --pass dx" \
 "300 bench12.log python bench.py --steps 20 --warmup 5"
