#!/bin/bash
# Kernel-purity profiles (rocprofv3 --kernel-trace) of every GPU training
# workload: ResNet-50 b1024 (bench.py), AlexNet b512, BERT-base, sonnx-BERT,
# the reference's mlp.conf / conv.conf through the config-driven Worker, and
# the fp32 MLP.  Summaries: gpurun_out/purity/<workload>.txt (+ .json).
#   tools/purity_all.sh [tag] [workloads...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r3}
shift
wl=${*:-"resnet50 alexnet bert bert_sonnx mlp_gpu mlp_conf conv_conf easgd rsync"}
out=gpurun_out/purity
mkdir -p $out
run() {  # name, steps, command...
  local name=$1 steps=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 420 rocprofv3 --kernel-trace -d $out/db_$name -o k --output-format rocpd -- "$@" \
    > $out/${name}_${tag}.log 2>&1 || { echo "FAILED $name ($?)"; tail -20 $out/${name}_${tag}.log; return 1; }
  local db
  db=$(find $out/db_$name -name '*.db' | head -1)
  python3 tools/kernel_purity.py "$db" --workload "$name" --steps "$steps" --json $out/${name}_${tag}.json \
    > $out/${name}_${tag}.txt && head -30 $out/${name}_${tag}.txt
  rm -rf $out/db_$name
}
for w in $wl; do
  case $w in
    resnet50) run resnet50 6 python3 bench.py --steps 3 --warmup 3 --no-ps-parity || exit 1 ;;
    alexnet) run alexnet 5 python3 tools/bench_suite.py --which alexnet --steps 3 --warmup 2 || exit 1 ;;
    bert) run bert 5 python3 tools/bench_suite.py --which bert --steps 3 --warmup 2 || exit 1 ;;
    bert_sonnx) run bert_sonnx 5 python3 tools/bench_suite.py --which bert_sonnx --steps 3 --warmup 2 || exit 1 ;;
    mlp_gpu) run mlp_gpu 5 python3 tools/bench_suite.py --which mlp_gpu --steps 3 --warmup 2 || exit 1 ;;
    mlp_conf) run mlp_conf 20 python3 -m singa_amd --model_conf examples/mnist/mlp.conf --device gpu --synthetic \
      --train_steps 20 || exit 1 ;;
    easgd) run easgd 20 python3 tools/easgd_workload.py --ptype Elastic --steps 20 || exit 1 ;;
    rsync) run rsync 20 python3 tools/easgd_workload.py --ptype RandomSync --steps 20 || exit 1 ;;
    conv_conf) run conv_conf 20 python3 -m singa_amd --model_conf examples/mnist/conv.conf --device gpu --synthetic \
      --train_steps 20 || exit 1 ;;
  esac
done
