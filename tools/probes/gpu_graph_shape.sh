#!/bin/bash
# shape of the captured ResNet-50 step graph (node / edge counts, forks, joins,
# node types: ops.graph_info) and the host enqueue time with the own RCCL communicator (world of
# one, EWDML_FORCE_PG=1) against the local one, for the compressed and the dense exchange.
# Outputs under gpurun_out/graph_shape/.  Run through gpurun from the repo root.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/graph_shape
mkdir -p $out
run() {  # name env... -- args
  name=$1; shift
  env "$@" EWDML_GRAPH_DUMP=$out/$name.graph.json timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 200)) \
    bench.py --gpus 1 --preset resnet50_cifar --steps 6 --warmup 4 --no-extras $ARGS \
    > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; return 1; }
  rm -f $out/$name.graph.json.dot  # large; the JSON summary is kept
  python3 -c "import json; d=json.loads([l for l in open('$out/$name.json') if l.startswith('{')][-1]); import os; g=json.load(open('$out/$name.graph.json')) if os.path.exists('$out/$name.graph.json') else 'no dump (segmented)'; print('$name', d['value'], d['ms_per_step'], 'enq', d['host_enqueue_ms_per_step'], d['config']['comm'], d['config']['hip_graph'], g)"
}
for codec in "--compress none" ""; do
  ARGS="$codec"
  tag=$([ -n "$codec" ] && echo dense || echo topk)
  run ${tag}_local EWDML_X=0 || exit 1
  run ${tag}_rccl EWDML_FORCE_PG=1 || exit 1
  run ${tag}_rccl_nomix EWDML_FORCE_PG=1 NCCL_GRAPH_MIXING_SUPPORT=0 || exit 1
done
# segmented (the comm graphs beside the compute segments), dense and top-k, real communicator
for codec in "--compress none" ""; do
  ARGS="$codec --hip-graph segmented"
  tag=$([ -n "$codec" ] && echo dense || echo topk)
  run ${tag}_rccl_seg EWDML_FORCE_PG=1 || exit 1
done
