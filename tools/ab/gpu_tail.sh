#!/bin/bash
# Fused VGG classifier tail: tests, then bench A/B against head.hip's per-Linear kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_head_tail.py tests/kernels/test_nn_kernels.py -q --timeout 120 --timeout-method thread -k "tail or head" \
    > gpurun_out/tail_tests.log 2>&1
rc=$?; tail -2 gpurun_out/tail_tests.log; grep -E "^E |FAILED" gpurun_out/tail_tests.log | head -10
[ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 3 "tail||--no-extras" "perlinear|EWDML_HEAD_TAIL=0|--no-extras" || exit 1
