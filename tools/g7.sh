cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof256 -o r50 --output-format rocpd -- python3 bench.py --steps 15 --warmup 3 --batch 256 > gpurun_out/prof256.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof512 -o r50 --output-format rocpd -- python3 bench.py --steps 10 --warmup 3 --batch 512 > gpurun_out/prof512.log 2>&1
echo rc=$?
