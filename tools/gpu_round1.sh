#!/bin/bash
# First GPU validation: kernel numerics vs oracle, smoke, short bench.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -m pytest tests/kernels -x -q -m gpu > gpurun_out/kern.log 2>&1 || { echo "kernel tests failed"; tail -40 gpurun_out/kern.log; exit 1; }
tail -3 gpurun_out/kern.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --compress none > gpurun_out/bench_dense.log 2>&1 || { echo "bench dense failed"; tail -40 gpurun_out/bench_dense.log; exit 1; }
tail -2 gpurun_out/bench_dense.log
