#!/bin/bash
# round 5: VGG conv tests (fp64 batch 32, in-situ batch 64) + Winograd F(4x4) on the 8x8 layers A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/kernels/test_conv_f32.py -v --timeout 200 --timeout-method thread \
    -k "vgg11 or smallmap" > gpurun_out/r5a_tests.log 2>&1
rc=$?; grep -E "FAILED|Error:|passed|failed" gpurun_out/r5a_tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
bash tools/gpurun_suite.sh ab 2 "m2||--no-extras" "m4_8x8|EWDML_WINO_M4_MIN_TILES=512|--no-extras" || exit 1
