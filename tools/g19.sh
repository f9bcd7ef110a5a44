cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_step.sh \
 "300 gputests_bn2.log python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'bn or batchnorm' --timeout 300 --timeout-method thread" \
 "300 bench_g.log python bench.py --steps 30 --warmup 10" \
 "300 bench_eager.log python bench.py --steps 30 --warmup 10 --no-graph" || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof10 -o r50 --output-format rocpd -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof10.log 2>&1
echo rc=$?
