#!/bin/bash
# BN finalize by the small-map backward's last row tiles: tests, then the step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_conv_f32.py -q --timeout 200 --timeout-method thread \
    -k "rides or smallmap or vgg11" > gpurun_out/smride_tests.log 2>&1
rc=$?; tail -3 gpurun_out/smride_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 3 "ride||--no-extras" "noride|EWDML_BN_FIN_RIDE=0|--no-extras" || exit 1
bash tools/gpurun_suite.sh prof vgg_smride "--no-extras" > /dev/null || exit 1
grep -E "finalize|per step|k_sm_bwd" gpurun_out/prof_vgg_smride.txt | head -8
