#!/bin/bash
# BN apply coefficients in registers (EWDML_BN_REGS=1) vs the LDS copy: BN tests, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
EWDML_BN_REGS=1 timeout -k 10 600 python -u -m pytest tests/kernels -q --timeout 200 --timeout-method thread \
    -k "bn or vgg11 or resnet" > gpurun_out/bnregs_tests.log 2>&1
rc=$?; tail -2 gpurun_out/bnregs_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 2 "regs|EWDML_BN_REGS=1|--no-extras" "lds||--no-extras" \
    "r50_regs|EWDML_BN_REGS=1|--preset resnet50_cifar --no-extras" "r50_lds||--preset resnet50_cifar --no-extras" || exit 1
