#!/bin/bash
# round 6: sanity of the rebuilt in-tree extension
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 t_9p.log python -u -m pytest tests/test_generic_gemm_gpu.py tests/test_bert_fused_gpu.py tests/test_fattn_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q "failed" gpurun_out/t_9p.log && exit 1
tools/gpu_step.sh "200 p_smoke.log python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" "200 p_bert.log python bench.py --model bert --steps 30 --warmup 5" "200 p_r50.log python bench.py" || exit $?
