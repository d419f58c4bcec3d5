#!/bin/bash
# BN backward finalisation riding in the weight-gradient GEMM (EWDML_BN_FIN_RIDE): tests, trace, A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/kernels/test_conv_f32.py -q --timeout 120 --timeout-method thread \
    -k "bn_finalize or bn_backward_sums or vgg11 or lazy or resnet18" > gpurun_out/finride_tests.log 2>&1
rc=$?; tail -3 gpurun_out/finride_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh prof vgg_ride "--no-extras" > /dev/null || exit 1
grep -E "finalize|per step|k_cf_gemm<2" gpurun_out/prof_vgg_ride.txt | head -12
bash tools/gpurun_suite.sh ab 2 "ride||--no-extras" "noride|EWDML_BN_FIN_RIDE=0|--no-extras" || exit 1
bash tools/gpurun_suite.sh ab 1 "r50ride||--preset resnet50_cifar --no-extras" "r50noride|EWDML_BN_FIN_RIDE=0|--preset resnet50_cifar --no-extras" || exit 1
