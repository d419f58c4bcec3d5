#!/bin/bash
# 2x2-map dense GEMMs + fused-select hardening: kernel tests, the VGG-11 step tests, then an
# interleaved A/B against Winograd (EWDML_SMALLMAP=0) and a kernel trace of the new step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_conv_f32.py -v --timeout 120 --timeout-method thread -k smallmap > gpurun_out/sm_unit.log 2>&1; grep -E "PASSED|FAILED|Error:" gpurun_out/sm_unit.log | head -20
timeout -k 10 600 python -u -m pytest tests/kernels/test_conv_f32.py tests/kernels/test_hip_codecs.py -v --timeout 120 \
    --timeout-method thread -k "smallmap or vgg11 or lazy_bn or deterministic or lookback or fused_select or predictive" > gpurun_out/sm_tests.log 2>&1
rc=$?; grep -E "FAILED|Error:|passed|failed" gpurun_out/sm_tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1   # 1 = test failures (read the log); anything else: stop
bash tools/gpurun_suite.sh ab 2 "sm||--no-extras" "wino|EWDML_SMALLMAP=0|--no-extras" || exit 1
bash tools/gpurun_suite.sh prof sm "--no-extras" || exit 1
