tools/gpu_step.sh \
 "300 bnbench.log python tools/bench_bn.py --out gpurun_out/bn_bench.jsonl" \
 "600 gputests_bn.log python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'bn or batchnorm' --timeout 300 --timeout-method thread" \
 "600 bench_ur2.log python bench.py --steps 30 --warmup 10"
