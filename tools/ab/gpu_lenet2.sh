#!/bin/bash
# Fused LeNet step: kernel tests, bench A/B against the module path, kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_lenet_fused.py -v --timeout 120 --timeout-method thread \
    > gpurun_out/lenet_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/lenet_tests.log | tail -12
[ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 2 "fused||--preset lenet --no-extras" "module|EWDML_LENET_FUSED=0|--preset lenet --no-extras" || exit 1
bash tools/gpurun_suite.sh prof lenet_fused "--preset lenet --no-extras" || exit 1
