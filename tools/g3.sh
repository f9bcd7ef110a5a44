cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM TCC_HIT_sum TCC_MISS_sum"
set -e
for cfg in "--C 256 --H 14 --K 256 --R 3 --s 1" "--C 64 --H 56 --K 256 --R 1 --s 1"; do
 for ps in fwd wgrad; do
  tag=$(echo "$cfg $ps" | tr -d ' -')
  timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmc/$tag/p1 -o p1 --output-format rocpd -- python3 tools/conv_one.py $cfg --pass $ps --iters 5 > gpurun_out/pmc_$tag.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmc/$tag/p2 -o p2 --output-format rocpd -- python3 tools/conv_one.py $cfg --pass $ps --iters 5 >> gpurun_out/pmc_$tag.log 2>&1
 done
done
echo pmc done
