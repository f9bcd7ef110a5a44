cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof12 -o r50 --output-format rocpd -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof12.log 2>&1
echo rc=$?
