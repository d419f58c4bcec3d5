#!/bin/bash
# fused NHWC BN/ReLU/pool kernels: numerics, full GPU suite, A/B vs the NCHW module path
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
timeout -k 10 300 python -m pytest tests/kernels/test_nn_kernels.py -x -q -s > gpurun_out/nn_tests.log 2>&1 || { tail -60 gpurun_out/nn_tests.log; exit 1; }
tail -3 gpurun_out/nn_tests.log
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
bash tools/ab.sh 2 "nchw_mod||--layout nchw --fused-nn off" "nhwc_fused||--layout auto" "nhwc_mod||--layout nhwc --fused-nn off"
