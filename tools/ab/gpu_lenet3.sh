#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_lenet_fused.py -q --timeout 120 --timeout-method thread \
    > gpurun_out/lenet_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lenet_tests.log; grep -E "Error" gpurun_out/lenet_tests.log | head -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u tools/probes/lenet_probe.py || exit 1
bash tools/gpurun_suite.sh ab 2 "fused||--preset lenet --no-extras" || exit 1
bash tools/gpurun_suite.sh prof lenet_fused "--preset lenet --no-extras" || exit 1
