#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof3
export TMPDIR=/tmp EWDML_PROF_GAP=1
for v in "topk_g128_b16:--bucket-mb 16" "topk_g128_b64:--bucket-mb 64" "dense_g128:--compress none"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_$name -o run -- python3 bench.py --steps 20 --warmup 6 $args > gpurun_out/prof3/$name.log 2>&1 || { echo "prof $name failed"; tail -30 gpurun_out/prof3/$name.log; exit 1; }
  python3 tools/prof_summarize.py /tmp/p_$name gpurun_out/prof3/${name}_summary.txt --steps 20 > /dev/null || exit 1
  rm -rf /tmp/p_$name
done
unset EWDML_PROF_GAP
for args in "--bucket-mb 64" "--bucket-mb 4" "--bucket-mb 8" "--bucket-mb 64 --hip-graph split"; do
  echo "== $args" >> gpurun_out/sweep3.log
  timeout -k 10 300 python bench.py --steps 30 --warmup 6 $args > /tmp/one.log 2>&1 || { echo "sweep failed: $args"; tail -30 /tmp/one.log; exit 1; }
  grep '^{' /tmp/one.log >> gpurun_out/sweep3.log
done
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest gpu rc=$?"; tail -5 gpurun_out/pytest_gpu.log
echo done
