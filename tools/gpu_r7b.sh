#!/bin/bash
# graph-default bench: the driver's exact command forms, eager opt-out, 2-rank gloo rehearsal, smoke
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh "300 d_default.log python bench.py" "200 d_k20.log python bench.py --gpus 1 --steps 20 --warmup 5" \
  "200 d_eager.log python bench.py --steps 20 --warmup 5 --eager" \
  "300 d_sl.log env SINGA_DIST_BACKEND=gloo python bench.py --gpus 2 --batch 128 --steps 3 --warmup 1 --no-ps-parity" \
  "200 d_smoke.log python -c 'import __graft_entry__ as g; g.smoke()'"
