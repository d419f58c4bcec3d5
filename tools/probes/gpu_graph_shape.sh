#!/bin/bash
# shape of the captured ResNet-50 step graph with the own RCCL communicator
# (world of one, EWDML_FORCE_PG=1) against the local one.  Writes DOT dumps and their summaries
# under gpurun_out/graph_shape/.  Run through gpurun from the repo root.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/graph_shape
mkdir -p $out
args="--preset resnet50_cifar --steps 6 --warmup 4 --no-extras ${EXTRA:-}"
EWDML_GRAPH_DUMP=/tmp/g_local.dot timeout -k 10 300 python bench.py $args > $out/local.json 2> $out/local.err \
  || { tail -20 $out/local.err; exit 1; }
EWDML_FORCE_PG=1 EWDML_GRAPH_DUMP=/tmp/g_rccl.dot timeout -k 10 300 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 1 $args \
  > $out/rccl.json 2> $out/rccl.err || { tail -20 $out/rccl.err; exit 1; }
# NCCL_GRAPH_MIXING_SUPPORT=0: the communicator does not join its internal stream to the caller's
# around captured collectives (fewer fork / join nodes)
NCCL_GRAPH_MIXING_SUPPORT=0 EWDML_FORCE_PG=1 EWDML_GRAPH_DUMP=/tmp/g_rccl_nomix.dot timeout -k 10 300 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29632 bench.py --gpus 1 $args > $out/rccl_nomix.json 2> $out/rccl_nomix.err \
  || { tail -20 $out/rccl_nomix.err; exit 1; }
python3 tools/probes/graph_shape.py /tmp/g_local.dot /tmp/g_rccl.dot /tmp/g_rccl_nomix.dot \
  > $out/shape.txt || exit 1
for f in local rccl rccl_nomix; do
  python3 -c "import json,sys; d=json.loads([l for l in open('$out/$f.json') if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], 'enq', d['host_enqueue_ms_per_step'], d['config']['comm'], d['config']['hip_graph'])"
done
grep -v '^ *"' $out/shape.txt | head -5
python3 - <<'PY'
import re
for f in ("/tmp/g_local.dot", "/tmp/g_rccl.dot", "/tmp/g_rccl_nomix.dot"):
    t = open(f).read()
    print(f, "bytes", len(t))
    # node kinds by the label's first word
    kinds = {}
    for m in re.finditer(r'label="\{?\s*([A-Za-z_]+)', t):
        kinds[m.group(1)] = kinds.get(m.group(1), 0) + 1
    print(sorted(kinds.items(), key=lambda kv: -kv[1])[:12])
PY
head -c 3000 /tmp/g_rccl.dot > $out/rccl_head.dot
