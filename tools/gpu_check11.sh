#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "vgg||" "r50c||--preset resnet50_cifar"
bash tools/gpu_profile8.sh
