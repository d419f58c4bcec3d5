#!/bin/bash
# GPU validation pass: every GPU test, smoke(), the default bench twice, the dense baseline and
# the other BASELINE presets.  Each GPU step has its own time limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for p in ${PRESETS:-vgg11 vgg11}; do
  timeout -k 10 300 python bench.py --preset $p > gpurun_out/bench_$p.json 2> gpurun_out/bench_err.log \
      || { tail -30 gpurun_out/bench_err.log; exit 1; }
  tail -1 gpurun_out/bench_$p.json
done
