#!/bin/bash
# In-launch split-K reduction (EWDML_CF_INRED): tests, then A/B on VGG-11 and ResNet-50 CIFAR.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_conv_f32.py -q --timeout 200 --timeout-method thread \
    > gpurun_out/inred_tests.log 2>&1
rc=$?; tail -3 gpurun_out/inred_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 2 "inred||--no-extras" "sep|EWDML_CF_INRED=0|--no-extras" \
    "r50_inred||--preset resnet50_cifar --no-extras" "r50_sep|EWDML_CF_INRED=0|--preset resnet50_cifar --no-extras" || exit 1
