#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
rm -f gpurun_out/ab.log
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/bench_vgg_$i.json 2> gpurun_out/bench_err.log || { tail -20 gpurun_out/bench_err.log; exit 1; }; tail -1 gpurun_out/bench_vgg_$i.json; done
