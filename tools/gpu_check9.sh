#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/kernels/test_nn_kernels.py tests/kernels/test_make_batch.py -x -q > gpurun_out/new_tests.log 2>&1 || { tail -60 gpurun_out/new_tests.log; exit 1; }
tail -2 gpurun_out/new_tests.log
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 1 "r50c_nchw_mod||--preset resnet50_cifar --layout nchw --fused-nn off" "r50c_fused||--preset resnet50_cifar" "vgg||"
bash tools/ab.sh 1 "r50i_nchw_mod||--preset resnet50_imagenet --layout nchw --fused-nn off" "r50i_fused||--preset resnet50_imagenet" "lenet||--preset lenet"
