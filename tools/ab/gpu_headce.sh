#!/bin/bash
# Cross-entropy riding in the last Linear (EWDML_HEAD_CE): tests, then A/B on VGG-11.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_head_ce.py tests/kernels/test_head_tail.py \
    "tests/e2e/test_gpu_train.py::test_own_rccl_communicator_matches_process_group" -q --timeout 200 \
    --timeout-method thread > gpurun_out/headce_tests.log 2>&1
rc=$?; tail -3 gpurun_out/headce_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 2 "ce||--no-extras" "noce|EWDML_HEAD_CE=0|--no-extras" || exit 1
