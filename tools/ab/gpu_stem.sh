#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_conv_f32.py -q --timeout 120 --timeout-method thread -k "stem" > gpurun_out/stem_tests.log 2>&1
rc=$?; tail -1 gpurun_out/stem_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh prof vgg_stem "--no-extras" > /dev/null || exit 1
grep -E "k_cf_stem|per step" gpurun_out/prof_vgg_stem.txt | head -5
bash tools/gpurun_suite.sh ab 2 "vgg||--no-extras" || exit 1
