#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/e2e/test_gpu_train.py -x -q > gpurun_out/e2e.log 2>&1 || { tail -40 gpurun_out/e2e.log; exit 1; }
tail -1 gpurun_out/e2e.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "vgg||" "r50c||--preset resnet50_cifar"
bash tools/gpu_profile8.sh
