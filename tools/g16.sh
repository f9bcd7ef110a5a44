tools/gpu_step.sh "600 suite.log python tools/bench_suite.py --which mlp_gpu,alexnet,bert,bert_sonnx --out gpurun_out/suite.jsonl"
