#!/bin/bash
# BN finalize with its per-channel operands loaded ahead of the partial sums: BN tests, bench, trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels -q -x --timeout 120 --timeout-method thread -k "bn or batchnorm or lenet" \
    > gpurun_out/fin_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fin_tests.log; grep -E "^E |FAILED" gpurun_out/fin_tests.log | head -8
[ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 2 "vgg||--no-extras" || exit 1
bash tools/gpurun_suite.sh prof vgg_fin "--no-extras" || exit 1
