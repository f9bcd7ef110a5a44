#!/bin/bash
# rocprofv3 kernel trace of the flagship step (bench.py, default config);
# the summary goes to gpurun_out/prof_<tag>.txt and the kernel-purity record
# to gpurun_out/purity_<tag>.json (copy both into profiles/).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-step}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o r50 --output-format rocpd -- python3 bench.py --steps 8 --warmup 3 --no-ps-parity > gpurun_out/prof_$tag.log 2>&1 || exit $?
db=$(find gpurun_out/prof_$tag -name '*.db' | head -1)
python3 tools/prof_summary.py "$db" --steps 11 > gpurun_out/prof_$tag.txt
python3 tools/kernel_purity.py "$db" --workload resnet50_b1024 --json gpurun_out/purity_$tag.json > gpurun_out/purity_$tag.txt
rm -rf gpurun_out/prof_$tag
