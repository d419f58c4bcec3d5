#!/bin/bash
# MFMA conv: numerics tests, then A/B vs MIOpen on the VGG-11 and ResNet-50 presets
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { tail -60 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 1 "vgg_hip|EWDML_CONV=hip|" "vgg_miopen|EWDML_CONV=miopen|" "r50c_hip|EWDML_CONV=hip|--preset resnet50_cifar" "r50c_miopen|EWDML_CONV=miopen|--preset resnet50_cifar" "r50i_hip|EWDML_CONV=hip|--preset resnet50_imagenet" "r50i_miopen|EWDML_CONV=miopen|--preset resnet50_imagenet"
