#!/bin/bash
# conv tests + interleaved A/B (2 rounds) of the three presets
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_conv.py tests/kernels/test_nn_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { tail -60 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "vgg_hip|EWDML_CONV=hip|" "r50c_hip|EWDML_CONV=hip|--preset resnet50_cifar" "r50i_hip|EWDML_CONV=hip|--preset resnet50_imagenet" "r50i_miopen|EWDML_CONV=miopen|--preset resnet50_imagenet"
