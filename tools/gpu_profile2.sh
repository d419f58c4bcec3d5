#!/bin/bash
# Timed-window kernel profiles of graph-mode steps + sweep (dense vs top-k, batch, layout, find).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp EWDML_PROF_GAP=1
for v in "topk_g128:--hip-graph full" "dense_g128:--hip-graph full --compress none" "topk_e128:--hip-graph off"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_$name -o run -- python3 bench.py --steps 20 --warmup 6 $args > gpurun_out/prof2/$name.log 2>&1 || { echo "prof $name failed"; tail -30 gpurun_out/prof2/$name.log; exit 1; }
  python3 tools/prof_summarize.py /tmp/p_$name gpurun_out/prof2/${name}_summary.txt --steps 20 > /dev/null || exit 1
  rm -rf /tmp/p_$name
done
unset EWDML_PROF_GAP
for args in "--hip-graph full --compress none" "--hip-graph full --batch-size 256" "--hip-graph full --batch-size 256 --compress none" "--hip-graph full --batch-size 512" "--hip-graph full --batch-size 512 --compress none" "--hip-graph full --channels-last" "--hip-graph full --batch-size 64" "--hip-graph full --batch-size 64 --compress none" "--hip-graph full --qsgd-bits 4"; do
  echo "== $args" >> gpurun_out/sweep2.log
  timeout -k 10 300 python bench.py --steps 30 --warmup 6 $args > /tmp/one.log 2>&1 || { echo "sweep failed: $args"; tail -30 /tmp/one.log; cp /tmp/one.log gpurun_out/sweep2_fail.log; exit 1; }
  grep '^{' /tmp/one.log >> gpurun_out/sweep2.log
done
echo "== benchmark off, full graph" >> gpurun_out/sweep2.log
EWDML_CUDNN_BENCHMARK=0 timeout -k 10 300 python bench.py --steps 30 --warmup 6 --hip-graph full > /tmp/one.log 2>&1 && grep '^{' /tmp/one.log >> gpurun_out/sweep2.log
echo done
