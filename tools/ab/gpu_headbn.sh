#!/bin/bash
# BN8 backward riding in the head's first Linear (EWDML_HEAD_BN): tests, then A/B on VGG-11.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_head_ce.py tests/kernels/test_head_tail.py \
    tests/kernels/test_conv_f32.py -k "head or tail or vgg11 or bn_finalize" -q --timeout 200 \
    --timeout-method thread > gpurun_out/headbn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/headbn_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 2 "bn||--no-extras" "nobn|EWDML_HEAD_BN=0|--no-extras" || exit 1
