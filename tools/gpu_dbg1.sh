#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
EWDML_FORCE_PG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 4 --warmup 4 --batch-size 64 --compress none > gpurun_out/dbg_none.log 2>&1; echo "rc=$?"
grep -v "^\s*frame\|^E  *frame" gpurun_out/dbg_none.log | head -40
