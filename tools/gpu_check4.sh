#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 800 python tools/debug_capture.py > gpurun_out/debug_capture.log 2>&1; echo "debug rc=$?"; cat gpurun_out/debug_capture.log | grep "=="
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest gpu rc=$?"; tail -5 gpurun_out/pytest_gpu.log
for args in "--bucket-mb 64" "--bucket-mb 64 --compress none" "--bucket-mb 16" "--bucket-mb 64 --batch-size 256" "--bucket-mb 64 --batch-size 256 --compress none"; do
  echo "== $args" >> gpurun_out/sweep4.log
  timeout -k 10 300 python bench.py --steps 30 --warmup 6 $args > /tmp/one.log 2>&1 || { echo "sweep failed: $args"; tail -30 /tmp/one.log; exit 1; }
  grep '^{' /tmp/one.log >> gpurun_out/sweep4.log
done
echo done
