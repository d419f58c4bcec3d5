#!/bin/bash
# Unrolled graph replays (bench --graph-unroll): bitwise test, then A/B on VGG-11 and LeNet.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/e2e/test_gpu_train.py -q --timeout 120 --timeout-method thread \
    -k "unrolled or graph_modes_match" > gpurun_out/unroll_tests.log 2>&1
rc=$?; tail -3 gpurun_out/unroll_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 2 "u1||--no-extras --graph-unroll 1" "u4||--no-extras --graph-unroll 4" \
    "u8||--no-extras --graph-unroll 8" || exit 1
bash tools/gpurun_suite.sh ab 2 "lenet_u1||--preset lenet --no-extras --graph-unroll 1" \
    "lenet_u4||--preset lenet --no-extras --graph-unroll 4" "lenet_u8||--preset lenet --no-extras --graph-unroll 8" || exit 1
