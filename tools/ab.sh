#!/bin/bash
# Interleaved A/B of bench variants on one box: variants x rounds, one JSON line each.
# usage: tools/ab.sh ROUNDS "NAME|ENV|ARGS" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    IFS='|' read -r name envs args <<< "$v"
    out=$(env $envs timeout -k 10 300 python bench.py --steps 40 --warmup 6 $args 2>/tmp/ab_err.log | grep '^{') || { echo "FAILED $name"; tail -20 /tmp/ab_err.log; exit 1; }
    echo "$name r$r $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ab.log
  done
done
