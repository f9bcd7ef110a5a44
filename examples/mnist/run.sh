#!/bin/bash
# Launch one process per GPU on this node (replaces the reference's ssh fan-out).
# usage: examples/mnist/run.sh [nproc] [model conf] [cluster conf]
N=${1:-2}
MODEL=${2:-examples/mnist/mlp.conf}
CLUSTER=${3:-examples/mnist/cluster.conf}
exec python -m singa_amd.launch --nproc "$N" -- --model_conf "$MODEL" --cluster_conf "$CLUSTER" "${@:4}"
