#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/kernels/test_nn_kernels.py -x -q > gpurun_out/nn_tests.log 2>&1 || { tail -60 gpurun_out/nn_tests.log; exit 1; }
tail -2 gpurun_out/nn_tests.log
bash tools/gpu_profile7.sh
