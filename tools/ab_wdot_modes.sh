cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2; do for v in 1 2 0; do SINGA_AMD_BN_WDOT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ps-parity > gpurun_out/ab_tmp.log 2>&1 || { tail -20 gpurun_out/ab_tmp.log; exit 1; }; echo "$i wdot=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_tmp.log)" | tee -a gpurun_out/ab_wdot3.txt; done; done
