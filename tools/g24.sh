cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11 -o r50 --output-format rocpd -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/prof11.log 2>&1
echo rc=$?
