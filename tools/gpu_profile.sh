#!/bin/bash
# Per-kernel profile of the flagship step + a batch/layout/graph sweep.  Raw traces are summarised
# on the box and deleted (gpurun copies back at most 64 MiB).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for v in "topk:" "dense:--compress none"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- python3 bench.py --steps 20 --warmup 5 $args > gpurun_out/prof/$name.log 2>&1 || { echo "prof $name failed"; tail -30 gpurun_out/prof/$name.log; exit 1; }
  python3 tools/prof_summarize.py /tmp/prof_$name gpurun_out/prof/${name}_summary.txt > /dev/null || exit 1
  find /tmp/prof_$name -name "*stats*.csv" -exec cp {} gpurun_out/prof/ \; 
  for f in gpurun_out/prof/*stats*.csv; do [ -f "$f" ] && mv "$f" "gpurun_out/prof/${name}_$(basename $f)"; done
done
for args in "--hip-graph split" "--hip-graph full" "--batch-size 256" "--batch-size 512" "--batch-size 128 --channels-last" "--batch-size 128 --no-overlap" "--batch-size 512 --compress none" "--batch-size 256 --hip-graph split" "--batch-size 512 --hip-graph split"; do
  echo "== $args" >> gpurun_out/sweep.log
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $args > /tmp/sweep_one.log 2>&1 || { echo "sweep failed: $args"; tail -30 /tmp/sweep_one.log; cp /tmp/sweep_one.log gpurun_out/sweep_fail.log; exit 1; }
  grep '^{' /tmp/sweep_one.log >> gpurun_out/sweep.log
done
echo "== forced RCCL PG (world 1), full graph" >> gpurun_out/sweep.log
EWDML_FORCE_PG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --hip-graph full > /tmp/pg.log 2>&1 || { echo "forced-PG full graph failed"; tail -30 /tmp/pg.log; cp /tmp/pg.log gpurun_out/pg_fail.log; exit 1; }
grep '^{' /tmp/pg.log >> gpurun_out/sweep.log
echo done
