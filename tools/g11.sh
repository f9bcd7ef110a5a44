cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof512b -o r50 --output-format rocpd -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof512b.log 2>&1
echo rc=$?
