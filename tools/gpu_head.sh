#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_nn_kernels.py tests/kernels/test_conv.py tests/e2e/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/head_tests.log 2>&1 || { tail -60 gpurun_out/head_tests.log; exit 1; }
tail -1 gpurun_out/head_tests.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "head_fused|EWDML_HEAD=fused|" "head_torch|EWDML_HEAD=torch|"
