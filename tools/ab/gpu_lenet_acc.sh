#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/e2e/test_gpu_accuracy.py tests/kernels/test_lenet_fused.py -v --timeout 300 --timeout-method thread -k "lenet" \
    > gpurun_out/lenet_acc.log 2>&1
grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/lenet_acc.log | tail -12
